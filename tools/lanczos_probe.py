"""Dev probe: the device Lanczos alone (DCGS2, 20 probes x 30 steps) on the sparse5
operator, 3 runs timed, for kernel traces of its basis passes (lz_dots / lz_update)
without the multi-shift CG beside it. usage: lanczos_probe.py [sparse4|sparse5]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data  # noqa: E402

CFG = {'sparse4': (256, 2, 0.005, 1e-3), 'sparse5': (64, 3, 0.02, 6e-4)}
name = sys.argv[1] if len(sys.argv) > 1 else 'sparse5'
g, d, rho, dens = CFG[name]
pts = _data.generate_points(g, d, True)
D = generate_correlation(pts, rho, 1.5, sparse=True, density=dens, device_resident=True)
sop = D.op
sop.lanczos(20, 30, 0)
for r in range(3):
    t0 = time.perf_counter()
    sop.lanczos(20, 30, 0)
    print('%s lanczos 20 x 30: %.2f ms' % (name, (time.perf_counter() - t0) * 1e3), flush=True)
