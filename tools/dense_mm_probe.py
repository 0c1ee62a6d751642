"""Dev probe: dense_mm_kernel (K X over a resident dense K, gpmi_sp_create_dense)
at N = grid^2 for several column counts; HBM fraction of the 8 n^2 bytes of K.
usage: dense_mm_probe.py [grid]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data, _hip  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
pts = _data.generate_points(grid, 2, True)
D = generate_correlation(pts, 0.1, 1.5, device_resident=True)
sop = _hip.SparseOperator.from_dense(D.op)
n = sop.n
for s in (1, 8, 16, 20, 32):
    ms = sop.bench_spmm(s, 20)
    gbs = 8.0 * n * n / (ms * 1e-3) / 1e9
    print('n=%d s=%2d  %.4f ms  %7.1f GB/s  %.3f of HBM' % (n, s, ms, gbs, gbs / 8000.0), flush=True)
