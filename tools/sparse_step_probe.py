"""Where the host time of one sparse bench step goes (cfg 4 / cfg 5): the step of
bench.sparse_measure, timed by phase (Lanczos call, Ritz nodes, quadratures,
multi-shift CG thread, lp), 10 steps after 3 warm-ups.
usage: python tools/sparse_step_probe.py [sparse4|sparse5]"""
import os
import sys
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]

import bench                                                        # noqa: E402
from gaussian_proc import generate_correlation, _data, _slq          # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation       # noqa: E402
from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms   # noqa: E402


def main():
    import torch
    torch.cuda.set_device(0)   # torch's HIP context first, as bench.py does
    cfg = sys.argv[1] if len(sys.argv) > 1 else 'sparse4'
    npts, dim, rho, nu, dens, nprobe, steps, neta = bench.SPARSE_CONFIGS[cfg]
    pts = _data.generate_points(npts, dim, True)
    z = _data.generate_data(pts, 0.2)
    X = _data.generate_basis_functions(pts, 2)
    n, m = X.shape
    D = generate_correlation(pts, rho, nu, sparse=True, density=dens, device=0,
                             device_resident=True)
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': nprobe, 'lanczos_degree': steps})
    th = _slq.min_ritz(op.slq_nodes())
    etas = numpy.logspace(-2, 2, neta) + max(0.0, -1.1 * th)
    op.sop.set_rhs(numpy.column_stack([X, z]))
    acc = {}

    def tick(k, t0):
        acc[k] = acc.get(k, 0.0) + time.perf_counter() - t0

    for it in range(13):
        if it == 3:
            acc.clear()
            torch.cuda.synchronize()
            T0 = time.perf_counter()
        t0 = time.perf_counter()
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(1) as ex:
            tm = time.perf_counter()
            fut = ex.submit(lambda: (op.sop.msgram(etas, None, 1e-6), time.perf_counter())[::-1])
            tick('pool+submit', tm)
            t1 = time.perf_counter()
            a, b = op.sop.lanczos(nprobe, steps, op.seed, probe_offset=0, orthogonalize=0)
            tick('lanczos call', t1)
            t1 = time.perf_counter()
            nodes = _slq.nodes(a, b)
            tick('ritz nodes', t1)
            t1 = time.perf_counter()
            for name in ('logdet', 'traceinv', 'traceinv2'):
                _slq.quadrature(nodes, etas, _slq.FUNCS[name], check=False)
            tick('quadratures', t1)
            t1 = time.perf_counter()
            tdone, G = fut.result()
            tick('wait for CG', t1)
            acc['CG done after step start'] = acc.get('CG done after step start', 0.0) + tdone - t0
        t1 = time.perf_counter()
        ld = n * _slq.quadrature(nodes, etas, numpy.log, check=False).mean(axis=0)
        [_lp_from_terms(n, m, 1.0, l, g) for l, g in zip(ld, G)]
        tick('lp', t1)
        tick('step', t0)
    torch.cuda.synchronize()
    total = time.perf_counter() - T0
    print('%s: %.3f ms per step over 10' % (cfg, total / 10 * 1e3))
    for k, v in acc.items():
        print('  %-26s %8.3f ms' % (k, v / 10 * 1e3))


if __name__ == '__main__':
    main()
