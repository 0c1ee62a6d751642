"""Dev probe: the band reduction at N = 16384 cold, then right after ~10 s of dense
64-eta Cholesky batches (the bench's order), to separate the chip's state under
sustained fp64 MFMA load from the reduction itself. Argument dense-first: allocate the dense
workspaces before the band (the bench's allocation order); dense-first8: also run
a batch of 8 first (the dense operator then holds a second stream)."""
import os
import sys
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

pts = _data.generate_points(128, 2, True)
z = _data.generate_data(pts, 0.2)
X = _data.generate_basis_functions(pts, 2)
D = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=64)
etas = numpy.logspace(-3, 3, 64)
if len(sys.argv) > 1 and sys.argv[1].startswith('dense-first'):
    # the bench's order: the dense batch-64 workspaces exist before the band is made
    dense = MixedCorrelation(D)
    dense.loglik_terms(etas, X, z)
    if sys.argv[1] == 'dense-first8':   # a batch of 8: the dense op's second stream
        dense.loglik_terms(etas[:8], X, z)
band = MixedCorrelation(D, imate_method='eigenvalue')
b = band.band()
for r in range(3):
    band.refresh_band(X, z)
    print('cold refresh %d: %.1f ms' % (r, b.last_timing()['reduce_ms']), flush=True)
dense = MixedCorrelation(D)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 10.0:
    dense.loglik_terms(etas, X, z)
for r in range(3):
    band.refresh_band(X, z)
    print('after dense refresh %d: %.1f ms' % (r, b.last_timing()['reduce_ms']), flush=True)
time.sleep(10.0)
band.refresh_band(X, z)
print('after 10 s idle: %.1f ms' % b.last_timing()['reduce_ms'], flush=True)
