"""Dev probe: SpMM kernels per width on the bench's sparse configs (sparse4: 2D
N=65536, sparse5: 3D N=262144), per GPMI_SPMM_* setting (read at every launch).
usage: spmm_probe.py [sparse4|sparse5 ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data  # noqa: E402

CFG = {'sparse4': (256, 2, 0.005, 1e-3), 'sparse5': (64, 3, 0.02, 6e-4)}
SETTINGS = [('pair/gather', {'GPMI_SPMM_WING': '0', 'GPMI_SPMM_WINDOW': '0'}),
            ('window (old)', {'GPMI_SPMM_WING': '0'}),
            ('wing', {})]
for name in sys.argv[1:] or ['sparse5', 'sparse4']:
    g, d, rho, dens = CFG[name]
    pts = _data.generate_points(g, d, True)
    D = generate_correlation(pts, rho, 1.5, sparse=True, density=dens, device_resident=True)
    sop = D.op
    n, nnz = sop.n, sop.nnz
    for s in (20, 12, 11):
        alg = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n * s
        for label, env in SETTINGS:
            keep = {k: os.environ.get(k) for k in ('GPMI_SPMM_WING', 'GPMI_SPMM_WINDOW')}
            os.environ.update(env)
            ms = sop.bench_spmm(s, 20)
            kern = sop.spmm_kernel(s)
            for k, v in keep.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            print('%s s=%2d %-13s %-22s %8.1f us  %.3f of HBM' % (
                name, s, label, kern, ms * 1e3, alg / (ms * 1e-3) / 8e12), flush=True)
