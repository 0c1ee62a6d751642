"""Dev probe: band likelihood-term call time at N = 16384 (one band reduction),
sequential band_chol_kernel vs block cyclic reduction (GPMI_BAND_BCR), for
1 / 8 / 64 eta per call (device time, HIP events)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
import numpy  # noqa: E402
from gaussian_proc import generate_correlation, _data  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
pts = _data.generate_points(grid, 2, True)
z = _data.generate_data(pts, 0.2)
X = _data.generate_basis_functions(pts, 2)
D = generate_correlation(pts, 0.1, 1.5, device_resident=True)
op = MixedCorrelation(D, imate_method='eigenvalue')
b = op.band()
grid_eta = numpy.logspace(-3, 3, 64)
ref = None
for k in (1, 8, 16, 64):
    etas = grid_eta[:k]
    op.loglik_terms(etas, X, z)
    ts = []
    for _ in range(3):
        ld, G = op.loglik_terms(etas, X, z)
        ts.append(b.last_timing()['loglik_ms'])
    print('%s eta %2d: %.3f ms (device), logdet[0] %.15e' % (os.environ.get('GPMI_BAND_BCR', '0'),
                                                           k, min(ts), ld[0]), flush=True)
for k in (1, 8, 64):
    etas = grid_eta[:k]
    op._der_cache = None
    op.der_terms(etas, X, z)
    ts = []
    for _ in range(3):
        op._der_cache = None
        op.der_terms(etas, X, z)
        ts.append(b.der_ms())
    print('%s der eta %2d: %.3f ms (device)' % (os.environ.get('GPMI_BAND_BCR', '2'), k, min(ts)),
          flush=True)
