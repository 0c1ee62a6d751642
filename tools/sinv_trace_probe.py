"""Dev probe (round 6): the one-eta derivative call of trust-exact's Jacobian /
Hessian on the 'eigenvalue' operator (der_terms with traceinv=2: the cyclic-reduction
factor, G2 / G3, the selected inversion and its eta-tangent) at config 3, for
kernel traces (rocprofv3 --kernel-trace --stats). One band reduction, then `reps`
calls at eta = 1 (and `reps` at 64 etas).  usage: sinv_trace_probe.py [grid reps]"""
import os
import sys
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
pts = _data.generate_points(grid, 2, True)
z = _data.generate_data(pts, 0.2)
X = _data.generate_basis_functions(pts, 2)
D = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=1)
op = MixedCorrelation(D, imate_method='eigenvalue')
b = op.band()
b.set_rhs(numpy.column_stack([X, z]))
for want in (1, 2):
    b.der_terms([1.0], traceinv=want)
    t0 = time.perf_counter()
    for _ in range(reps):
        b.der_terms([1.0], traceinv=want)
    print('der_terms 1 eta traceinv=%d: %.3f ms per call (sinv %.3f ms)'
          % (want, (time.perf_counter() - t0) / reps * 1e3, b.sinv_ms()), flush=True)
etas = numpy.logspace(-3, 3, 64)
for want in (1, 2):
    b.der_terms(etas, traceinv=want)
    t0 = time.perf_counter()
    for _ in range(reps):
        b.der_terms(etas, traceinv=want)
    print('der_terms 64 eta traceinv=%d: %.3f ms per call (sinv %.3f ms)'
          % (want, (time.perf_counter() - t0) / reps * 1e3, b.sinv_ms()), flush=True)
