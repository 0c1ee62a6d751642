"""Dev probe (round 6): traceinv of exponent 2 on the 'eigenvalue' operator at
config 3 (N = grid^2, default 128^2 = 16384) by the eta-tangent of the selected
inversion (gpmi_band_traceinv2), against the eigenvalue sums it replaces:
  * device ms of traceinv(eta, 1) and (eta, 1 + 2) for 1 / 8 / 64 etas;
  * der_terms(traceinv=1) and (traceinv=2) wall ms for one eta (the Jacobian and
    Hessian calls of trust-exact);
  * tr1 / tr2 against the device eigenvalue sums at three etas;
  * the direct and profiled optimizers (bench.optimizer_timing): wall s and the
    number of eigenvalue calls.
usage: trace2_probe.py [grid]"""
import json
import os
import sys
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
import torch  # noqa: E402

torch.cuda.set_device(0)
from gaussian_proc import generate_correlation, _data  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402
import bench  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
pts = _data.generate_points(grid, 2, True)
z = _data.generate_data(pts, 0.2)
X = _data.generate_basis_functions(pts, 2)
D = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=1)
out = {'n': int(X.shape[0])}

op = MixedCorrelation(D, imate_method='eigenvalue')
b = op.band()
b.set_rhs(numpy.column_stack([X, z]))
out['reduce_ms'] = b.last_timing()['reduce_ms']
for ne in (1, 8, 64):
    etas = numpy.logspace(-3, 3, ne) if ne > 1 else numpy.array([1.0])
    r = {}
    for p in (1, 2):
        b.traceinv(etas, p)   # warm (allocation)
        t0 = time.perf_counter()
        b.traceinv(etas, p)
        r['exp%d_wall_ms' % p] = round((time.perf_counter() - t0) * 1e3, 3)
        r['exp%d_sinv_ms' % p] = round(b.sinv_ms(), 3)
    out['traceinv_%d_eta' % ne] = r
    print(ne, r, flush=True)
for want in (True, 2):
    b.der_terms([1.0], traceinv=want)
    t0 = time.perf_counter()
    b.der_terms([1.0], traceinv=want)
    out['der_terms_1eta_traceinv%s_wall_ms' % int(want)] = round((time.perf_counter() - t0) * 1e3,
                                                                3)
etas = numpy.array([1e-3, 1.0, 100.0])
tr1, _ = b.traceinv(etas, 1)
tr2, _ = b.traceinv(etas, 2)
t0 = time.perf_counter()
lam = op.eigenvalues()
out['eigenvalues_ms'] = round((time.perf_counter() - t0) * 1e3, 1)
e1 = numpy.array([numpy.sum(1.0 / (lam + e)) for e in etas])
e2 = numpy.array([numpy.sum((lam + e) ** -2.0) for e in etas])
out['tr1_rel_diff_vs_eigenvalues'] = float(numpy.max(numpy.abs(tr1 - e1) / e1))
out['tr2_rel_diff_vs_eigenvalues'] = float(numpy.max(numpy.abs(tr2 - e2) / e2))
print(out, flush=True)
b.close()
out['optimizer'] = bench.optimizer_timing(D, X, z)
print(json.dumps(out, indent=1))
