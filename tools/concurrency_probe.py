"""Probe: do two independent batched factorizations on two HIP streams overlap?

Runs the N=16384 workload as (a) one operator, batch 8, sequentially and
(b) two operators (own streams), batch 4 each, driven from two host threads
(ctypes releases the GIL). Prints evals/s for both.
"""
import os
import sys
import threading
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]

from gaussian_proc import generate_correlation, _data          # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402


def main():
    grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    pts = _data.generate_points(grid, 2, True)
    z = _data.generate_data(pts, 0.2)
    X = _data.generate_basis_functions(pts, 2)
    etas = numpy.logspace(-3, 3, 64)
    D8 = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=8)
    op8 = MixedCorrelation(D8)
    op8.loglik_terms(etas[:8], X, z)
    t0 = time.perf_counter()
    for r in range(reps):
        op8.loglik_terms(etas[8 * r % 64:8 * r % 64 + 8], X, z)
    t8 = time.perf_counter() - t0
    print('single op batch 8: %.2f evals/s' % (8 * reps / t8), flush=True)
    del op8, D8
    ops = []
    for _ in range(2):
        D = generate_correlation(pts, 0.1, 1.5, device_resident=True, max_batch=4)
        ops.append(MixedCorrelation(D))
        ops[-1].loglik_terms(etas[:4], X, z)

    def run(op, off):
        for r in range(reps):
            op.loglik_terms(etas[off:off + 4], X, z)

    th = [threading.Thread(target=run, args=(ops[i], 4 * i)) for i in range(2)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    t2 = time.perf_counter() - t0
    print('two ops x batch 4 concurrently: %.2f evals/s' % (8 * reps / t2), flush=True)
    t0 = time.perf_counter()
    for r in range(reps):
        ops[0].loglik_terms(etas[:4], X, z)
    t1 = time.perf_counter() - t0
    print('single op batch 4: %.2f evals/s' % (4 * reps / t1), flush=True)


if __name__ == '__main__':
    main()
