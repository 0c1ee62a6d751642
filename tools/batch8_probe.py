"""Dev probe: the dense path at small batches (the per-rank block of a strong-scaled
64-eta curve: 8 eta at N = 8, 16 at N = 4) per schedule knob: outer panel width
(set_outer), look-ahead, and GPMI_GROUPS (1: one stream; 2: batch halves on two
streams, the default for <= 32). usage: batch8_probe.py [grid]"""
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
D = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=16)
op = MixedCorrelation(D)
op.set_rhs(X, z)
etas = numpy.logspace(-3, 3, 64)
n = X.shape[0]
fl = n ** 3 / 3.0
for nb in (8, 16):
    for outer in (8, 12, 16, 24):
        op.op.set_outer(outer)
        op.loglik_terms(etas[:nb], X, z)
        ts = []
        for r in range(3):
            t0 = time.perf_counter()
            op.loglik_terms(etas[8 * r:8 * r + nb], X, z)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        print('batch %2d outer %2d groups %s: %.1f ms  %.2f evals/s  %.3f of 78.6 (n^3/3)'
              % (nb, outer, os.environ.get('GPMI_GROUPS', 'auto'), t * 1e3, nb / t,
                 nb * fl / t / 78.6e12), flush=True)
