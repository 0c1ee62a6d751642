"""Dev probe (round 6): the per-rank device work of the sparse configs' N-rank line
on ONE GPU, to state the expected N = 8 step without an 8-GPU node:
rank 0's share of a step is the Lanczos of its probe shard (sweep.shard over the
20 probes) beside the multi-shift CG of its right-hand-side column shard (over the
11 columns of [X z], every eta), exactly the two device calls
sweep.slq_gram_sweep makes on a rank (the all-gathers move <= 40 KB). Times the
two together (the CG on its worker thread, as the sweep) for world = 1, 2, 4, 8.
usage: shard_probe.py [sparse4|sparse5] [reps]"""
import json
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
from gaussian_proc.sweep import shard, _cg_worker  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else 'sparse5'
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
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
out = {'config': config, 'probes': nprobe, 'columns': R.shape[1], 'by_world': {}}
for world in (1, 2, 4, 8):
    plo, phi, _ = shard(nprobe, world, 0)
    clo, chi, _ = shard(R.shape[1], world, 0)
    cols = None if world == 1 else (clo, chi)

    def step():
        fut = ex.submit(op.sop.msgram, etas, None, 1e-6, None, cols)
        op.sop.lanczos(phi - plo, steps, op.seed, probe_offset=plo,
                       orthogonalize=op.orthogonalize)
        fut.result()

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    out['by_world'][str(world)] = {'rank0_probes': phi - plo, 'rank0_columns': chi - clo,
                                   'rank0_step_ms': round(ms, 3)}
    print(world, out['by_world'][str(world)], flush=True)
print(json.dumps(out, indent=1))
