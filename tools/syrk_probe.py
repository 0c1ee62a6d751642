"""Dev probe: time one batched factorization call (N=16384, 16 etas) and print the
per-class SYRK timing (GPMI_SYRK_TRACE=1). Works with experiment builds whose
numerics are deliberately wrong (GPMI_LIB_VARIANT): a non-SPD error is ignored."""
import os
import sys
import time

import numpy

sys.path[:0] = ['.', 'gaussian-process-param-estimation_amd']
os.environ.setdefault('GPMI_SYRK_TRACE', '1')
from gaussian_proc import _hip  # noqa: E402
from oracle import data  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
pts = data.generate_points(grid, 2, True)
op = _hip.Operator(pts.shape[0], device=0, max_batch=B)
op.assemble_matern(pts, 0.1, 1.5)
rhs = numpy.ones((pts.shape[0], 7))
op.set_rhs(rhs)
etas = numpy.logspace(-1, 1, B)
for rep in range(3):
    op.set_timing(rep > 0)
    t0 = time.perf_counter()
    try:
        op.loglik_batch(etas)
    except Exception as e:   # noqa: BLE001
        print('ignored:', str(e)[:80], file=sys.stderr)
    dt = time.perf_counter() - t0
    if rep > 0:
        t = op.last_timing()
        print('rep %d wall %.1f ms  syrk %.1f ms  %.2f TF/s  total %.1f ms' % (
            rep, 1e3 * dt, t['syrk_ms'], t['syrk_flops'] / (t['syrk_ms'] * 1e-3) / 1e12,
            t['total_ms']), flush=True)
