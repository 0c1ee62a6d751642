"""Dev probe: band_chol_kernel device time for a batch of eta (after one band
reduction at N = grid^2); used with GPMI_LIB_VARIANT builds to price its loads."""
import os
import sys

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
neta = int(sys.argv[2]) if len(sys.argv) > 2 else 64
pts = _data.generate_points(grid, 2, True)
z = _data.generate_data(pts, 0.2)
X = _data.generate_basis_functions(pts, 2)
D = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=1)
op = MixedCorrelation(D, imate_method='eigenvalue')
b = op.band()
etas = numpy.logspace(-3, 3, neta)
for rep in range(3):
    try:
        op.loglik_terms(etas, X, z)
    except numpy.linalg.LinAlgError:
        pass
    print('loglik %d etas: %.2f ms' % (neta, b.last_timing()['loglik_ms']), flush=True)
for rep in range(2):
    try:
        op.der_terms(etas, X, z)
    except numpy.linalg.LinAlgError:
        pass
    op._der_cache = None
    print('der_terms %d etas: %.2f ms' % (neta, b.der_ms()), flush=True)
