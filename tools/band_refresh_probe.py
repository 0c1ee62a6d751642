"""Dev probe: band reductions at config 3 (N = grid^2, default 128^2 = 16384)
only, for kernel traces of the reduction (rocprofv3 --kernel-trace): one warm-up
reduction, then `reps` timed refreshes. usage: band_refresh_probe.py [grid reps nu]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

if os.environ.get('PROBE_TORCH') == '1':   # a torch HIP context beside ours (as bench.py)
    import torch
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
nu = float(sys.argv[3]) if len(sys.argv) > 3 else 1.5
pts = _data.generate_points(grid, 2, True)
D = generate_correlation(pts, 0.1, nu, device_resident=True)
op = MixedCorrelation(D, imate_method='eigenvalue')
b = op.band()
print('first reduce %.1f ms' % b.last_timing()['reduce_ms'], b.stats(), flush=True)
for r in range(reps):
    op.refresh_band()
    print('refresh %d: reduce %.1f ms' % (r, b.last_timing()['reduce_ms']), flush=True)
