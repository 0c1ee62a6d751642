"""Dev probe: the PCIe-inclusive cost of the drop-in boundary at N = grid^2.
(1) a host K handed to MixedCorrelation (one H2D copy of n^2 doubles per operator);
(2) one 64-eta dense call with host X, z in and host results out, against the same
call's device time; (3) points -> device assembly (K never crosses PCIe)."""
import os
import sys
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
pts = _data.generate_points(grid, 2, True)
z = _data.generate_data(pts, 0.2)
X = _data.generate_basis_functions(pts, 2)
n = pts.shape[0]
t0 = time.perf_counter()
D = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=1)
t1 = time.perf_counter()
print('assembly on device (points in, K resident): %.1f ms' % (1e3 * (t1 - t0)), flush=True)
K = D.to_host() if hasattr(D, 'to_host') else generate_correlation(pts, 0.1, 1.5)
for rep in range(2):
    t0 = time.perf_counter()
    op = MixedCorrelation(K, imate_method='cholesky')
    t1 = time.perf_counter()
    print('host K %.2f GB -> MixedCorrelation: %.1f ms (%.1f GB/s)' % (
        K.nbytes / 1e9, 1e3 * (t1 - t0), K.nbytes / 1e9 / (t1 - t0)), flush=True)
    del op
etas = numpy.logspace(-3, 3, 64)
D64 = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=64)
op = MixedCorrelation(D64)
op.op.set_outer(16)
op.set_rhs(X, z)
op.loglik_terms(etas, X, z)
op.op.set_timing(True)
t0 = time.perf_counter()
ld, G = op.loglik_terms(etas, X, z)
t1 = time.perf_counter()
tm = op.op.last_timing()
print('64-eta call: wall %.1f ms (host X, z in; logdet, Gram out), device %.1f ms' % (
    1e3 * (t1 - t0), tm['total_ms']), flush=True)
