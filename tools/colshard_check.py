"""Dev check (round 6): the multi-shift CG's column blocks (gpmi_sp_msgram_cols) against
the full block at a BASELINE sparse config, per block width: where (eta, row, column)
any difference or NaN sits, and the window SpMM of each width against the gather
kernel (GPMI_SPMM_WING=0 cannot switch per call: the SpMM is checked against scipy).
usage: colshard_check.py [config]"""
import os
import sys

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
import torch  # noqa: E402

torch.cuda.set_device(0)
import bench  # noqa: E402
from gaussian_proc import generate_correlation, _data, _slq  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else 'sparse4'
npts, dim, rho, nu, dens, nprobe, steps, neta = bench.SPARSE_CONFIGS[config]
points = _data.generate_points(npts, dim, True)
z = _data.generate_data(points, 0.2)
X = _data.generate_basis_functions(points, 2)
D = generate_correlation(points, rho, nu, sparse=True, density=dens, device_resident=True)
op = MixedCorrelation(D, imate_method='slq',
                      imate_options={'num_samples': nprobe, 'lanczos_degree': steps})
theta_min = _slq.min_ritz(op.slq_nodes())
etas = numpy.logspace(-2, 2, neta) + max(0.0, -1.1 * theta_min)
R = numpy.column_stack([X, z])
op.sop.set_rhs(R)
nc = R.shape[1]
Kc = op.sop.csr()
rng = numpy.random.RandomState(0)
for s in range(1, 21):
    Xs = rng.randn(Kc.shape[0], s)
    Y = op.sop.spmm(0.5, Xs)
    ref = Kc @ Xs + 0.5 * Xs
    err = numpy.abs(Y - ref).max() / numpy.abs(ref).max()
    print('spmm s=%2d kernel %s rel err %.2e' % (s, op.sop.spmm_kernel(s), err), flush=True)
Gfull = op.sop.msgram(etas, None, 1e-6)
print('full: nan', int(numpy.isnan(Gfull).sum()), 'shape', Gfull.shape, flush=True)
for a, b in ((0, 4), (4, 7), (0, 2), (2, 4), (4, 5), (5, 7), (6, 7), (0, 1)):
    if b > nc:
        continue
    G = op.sop.msgram(etas, None, 1e-6, None, (a, b))
    d = G - Gfull[:, :, a:b]
    bad = numpy.argwhere(~numpy.isfinite(G))
    print('cols [%d, %d): nan %d, max |diff| %.2e, first bad %s'
          % (a, b, int((~numpy.isfinite(G)).sum()), numpy.nanmax(numpy.abs(d)),
             bad[:3].tolist()), flush=True)
