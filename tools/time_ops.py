"""Wall-clock timing of single-eta operator calls on one GPU (dev tool):
factorization (logdet), traceinv exponent 1 and 2, at grid x grid points."""
import sys
import time

import numpy

sys.path[:0] = ['.', 'gaussian-process-param-estimation_amd']
import gaussian_proc  # noqa: E402
from oracle import data  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
pts = data.generate_points(grid, 2, True)
D = gaussian_proc.generate_correlation(pts, 0.1, 1.5, device_resident=True)
op = D.op
n = op.n
for rep in range(2):
    for eta in (0.5 + rep, ):
        t0 = time.perf_counter()
        ld = op.logdet(eta)
        t1 = time.perf_counter()
        t_1 = op.traceinv(eta, 1)
        t2 = time.perf_counter()
        t_2 = op.traceinv(eta, 2)
        t3 = time.perf_counter()
        fl = n ** 3 / 3.0
        print('n=%d eta=%g logdet %.1f ms | traceinv1 %.1f ms (%.1f TF/s) | traceinv2 +%.1f ms '
              '(%.1f TF/s) | ld=%.6f tr1=%.6e tr2=%.6e'
              % (n, eta, 1e3 * (t1 - t0), 1e3 * (t2 - t1), fl / (t2 - t1) / 1e12,
                 1e3 * (t3 - t2), fl / (t3 - t2) / 1e12, ld, t_1, t_2), flush=True)
