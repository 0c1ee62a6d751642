"""Dev probe (round 6): the multi-shift CG's batching at a BASELINE sparse config, one
call with GPMI_MS_TRACE=1 (each host read's prediction, the iterations launched past
the last column's stop), then the step's two device calls timed as in the sweep.
usage: ms_trace.py [sparse4|sparse5]"""
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
op.sop.msgram(etas, None, 1e-6)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    op.sop.msgram(etas, None, 1e-6)
    ms = (time.perf_counter() - t0) * 1e3
    print('msgram alone %.3f ms, iterations %d, segments %s'
          % (ms, op.sop.last_cg_iterations, op.sop.msgram_segments()), flush=True)
os.environ['GPMI_MS_TRACE'] = '1'
op.sop.msgram(etas, None, 1e-6)
sys.stderr.flush()
