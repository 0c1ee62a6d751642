"""Dev probe (round 6): the sparse step's two device calls (the multi-shift CG on its
worker thread, the probes' Lanczos on the main thread, as sweep.slq_gram_sweep runs
them) with the Lanczos started d ms after the CG (time.sleep, about 0.1 ms late): whether the
Lanczos costs the CG less beside its narrow, compacted phase than beside its first,
full-width iterations.   usage: overlap_probe.py [sparse4|sparse5] [reps]"""
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
from gaussian_proc.sweep import _cg_worker  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else 'sparse4'
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
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
ex = _cg_worker()


def lanczos():
    op.sop.lanczos(nprobe, steps, op.seed, probe_offset=0, orthogonalize=op.orthogonalize)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


print('cg alone %.3f ms, lanczos alone %.3f ms'
      % (timed(lambda: op.sop.msgram(etas, None, 1e-6)), timed(lanczos)), flush=True)
for d in (0.0, 0.25, 0.5, 0.75, 1.0, 1.25, 1.5):
    def step():
        fut = ex.submit(op.sop.msgram, etas, None, 1e-6)
        if d > 0:
            time.sleep(d * 1e-3)   # (releases the GIL: the CG's host loop runs meanwhile)
        lanczos()
        fut.result()
    print('lanczos after %.2f ms: step %.3f ms' % (d, timed(step)), flush=True)
