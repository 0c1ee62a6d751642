"""Dev probe (round 6): how the sparse step's two device calls scale with their
block width on one GPU, alone (no concurrency): the multi-shift CG over all 11
columns of [X z] against column blocks of it (gpmi_sp_msgram_cols), and the
Lanczos over 20 probes against probe blocks. If narrower blocks cost less than
their share, a single-GPU step could split them.  usage: split_probe.py [config]"""
import os
import sys
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
import torch  # noqa: E402

torch.cuda.set_device(0)
import bench  # noqa: E402
from gaussian_proc import generate_correlation, _data, _slq  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else 'sparse5'
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


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


Gfull = op.sop.msgram(etas, None, 1e-6)
print('msgram all %d columns: %.3f ms, %d iterations'
      % (nc, timed(lambda: op.sop.msgram(etas, None, 1e-6)), op.sop.last_cg_iterations),
      flush=True)
for parts in (2, 3, 4):
    bounds = numpy.linspace(0, nc, parts + 1).round().astype(int)
    tot, its = 0.0, []
    for a, b in zip(bounds[:-1], bounds[1:]):
        tot += timed(lambda: op.sop.msgram(etas, None, 1e-6, None, (int(a), int(b))))
        its.append(op.sop.last_cg_iterations)
    G = numpy.concatenate([op.sop.msgram(etas, None, 1e-6, None, (int(a), int(b)))
                           for a, b in zip(bounds[:-1], bounds[1:])], axis=2)
    print('msgram %d column blocks %s: %.3f ms summed, iterations %s, max |G - Gfull| %.2e'
          % (parts, list(bounds), tot, its, numpy.abs(G - Gfull).max()), flush=True)
for p in (20, 10, 5):
    ms = timed(lambda: op.sop.lanczos(p, steps, op.seed, probe_offset=0,
                                      orthogonalize=op.orthogonalize))
    print('lanczos %d probes: %.3f ms (x %d = %.3f ms for 20)' % (p, ms, 20 // p, ms * 20 // p),
          flush=True)
