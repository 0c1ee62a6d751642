"""Dev probe: band path timing at config 3 (N = grid^2, default 128^2 = 16384):
band reduction, Q^T R, and the banded-Cholesky likelihood terms for the 64-point
eta grid; logdet checked against the golden cfg3 values when N = 16384."""
import json
import os
import sys
import time

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
D = generate_correlation(pts, 0.1, 1.5, device_resident=True)
op = MixedCorrelation(D, imate_method='eigenvalue')
t0 = time.perf_counter()
b = op.band()
t1 = time.perf_counter()
print('band reduce: wall %.1f ms, device %.1f ms' % (1e3 * (t1 - t0), b.last_timing()['reduce_ms']),
      flush=True)
etas = numpy.logspace(-3, 3, neta)
for rep in range(3):
    t0 = time.perf_counter()
    ld, G = op.loglik_terms(etas, X, z)
    t1 = time.perf_counter()
    t = b.last_timing()
    print('rep %d: %d etas wall %.1f ms (rhs %.2f ms, loglik device %.2f ms)' % (
        rep, neta, 1e3 * (t1 - t0), t['rhs_ms'], t['loglik_ms']), flush=True)
if grid == 128:
    cfg = json.load(open(os.path.join(REPO, 'tests', 'golden', 'cfg3_big.json')))
    ld3, _ = op.loglik_terms(cfg['etas'], X, z)
    print('cfg3 logdet rel err', numpy.abs(ld3 - cfg['logdet']) / numpy.abs(cfg['logdet']))
# the reduction alone vs with Q^T [X z] applied alongside (bench band_mode's form)
for rhs in (False, True, False, True):
    if rhs:
        op.refresh_band(X, z)
    else:
        op.refresh_band()
    print('refresh%s: reduce %.1f ms' % (' with Q^T[X z]' if rhs else '', b.last_timing()['reduce_ms']),
          flush=True)
