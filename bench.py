#!/usr/bin/env python
"""Benchmark: log-likelihood evaluations / s on the N=16384 dense Matérn-3/2
covariance (BASELINE.json metric), one process per GPU.

A step = one block of ``--eta-per-rank`` (64) eta values per rank of the grid
logspace(-3, 3, max(64, N * 64)) (at N=1 exactly the 64-point cfg3 curve; at
N > 1 a finer grid over the same range, no eta repeated across ranks): one
batched device call factorizes
K + eta_b I (fp64 MFMA Cholesky, fused forward solve of [X | z], logdet and
Gram), the host forms the direct log-likelihood (sigma = 1, sigma0 = sqrt(eta)),
and ONE all-gather (RCCL over xGMI at N > 1) collects the [logdet, lp] curve.
K is assembled on each GPU from the points before the timed region (inputs
resident in HBM). Per-rank work is fixed: scaling "weak".

Launch: python bench.py [--gpus 1 --steps K --warmup W]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""

import argparse
import json
import os
import platform
import sys
import time

import numpy

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(REPO, 'gaussian-process-param-estimation_amd')
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

FP64_MFMA_PEAK_TFLOPS = 78.6    # MI355X fp64 matrix, dense (AMD spec)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--grid', type=int, default=128, help='points per axis (n = grid^2)')
    ap.add_argument('--nu', type=float, default=1.5)
    ap.add_argument('--eta-per-rank', type=int, default=64,
                    help='eta values factorized together per device call (one step); at '
                         'N=1 the default step is the whole 64-point eta curve')
    ap.add_argument('--outer', type=int, default=16, help='outer panel width / 128')
    ap.add_argument('--lookahead', type=int, default=0,
                    help='1: panel factorization on a second stream overlaps the bulk '
                         'trailing update; 0: one stream, in order')
    ap.add_argument('--config', default='dense', choices=['dense', 'sparse4', 'sparse5'],
                    help='dense: the headline N=16384 metric; sparse4/sparse5: BASELINE '
                         'configs 4 and 5 (tapered Matern, SLQ + CG)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-der', action='store_true',
                    help='skip the der1 eta-sweep measurement of the band mode')
    ap.add_argument('--no-band', action='store_true',
                    help='skip the band-mode (eigenvalue operator) measurement of the dense run')
    ap.add_argument('--band-etas', type=int, default=64,
                    help='band mode: eta values per rank per step (one reduction per step)')
    ap.add_argument('--no-timing', action='store_true',
                    help='skip the per-kernel HIP-event roofline timing')
    return ap.parse_args()


def pmc_traffic(outer, batch, kernel='gpmi::syrk_kernel'):
    """HBM-side bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary of this configuration (profiles/r*/pmc_traffic_outer{outer}_b{batch}.json,
    FETCH_SIZE and WRITE_SIZE collected in separate passes; FETCH_SIZE doubled
    for gfx950 wide streaming reads per MI355X_MICROARCH.md 'HBM'). PMC counters
    cannot be collected inside the timed run, hence the committed file; None
    when no summary matches."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*',
                                          'pmc_traffic_outer%d_b%d.json' % (outer, batch))))
    if not files:
        return None, None
    with open(files[-1]) as fh:
        k = json.load(fh)['kernels'].get(kernel)
    if not k:
        return None, None
    # per_dispatch_first: only the timed call's launches (the run's later
    # golden-logdet call is a smaller batch)
    pd = k.get('per_dispatch_first', k['per_dispatch'])
    return (2.0 * pd['FETCH_SIZE'] + pd['WRITE_SIZE']) * 1024.0, os.path.relpath(files[-1], REPO)


def pmc_traffic_sparse(config, kernel='gpmi::csr_spmm_kernel'):
    """HBM-side bytes per timed SpMM launch from the committed PMC summary of this
    sparse config (profiles/r*/pmc_traffic_{config}.json, per_dispatch_last = the
    bench's timed s=20 launches; FETCH_SIZE doubled as in pmc_traffic)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*',
                                          'pmc_traffic_%s.json' % config)))
    if not files:
        return None, None
    with open(files[-1]) as fh:
        k = json.load(fh)['kernels'].get(kernel)
    if not k or 'per_dispatch_last' not in k:
        return None, None
    pd = k['per_dispatch_last']
    return (2.0 * pd['FETCH_SIZE'] + pd['WRITE_SIZE']) * 1024.0, os.path.relpath(files[-1], REPO)


def cpu_baseline(points, z, X, nu, etas):
    """The reference's CPU call pattern, timed on this host (rank 0, N=1):
    Likelihood -> MixedCorrelation(imate_method='eigenvalue') -> per eval
    2 x scipy.linalg.solve(K + eta I, ., assume_a='pos') + O(n) eigen logdet
    (_direct_likelihood.py:59-71, mixed_correlation.py:239-299). Sample: ONE
    evaluation at the full N (the one-time eigh setup is excluded and reported
    separately as not timed). Uses the oracle restatement (kind 'port')."""
    from oracle import matern
    import scipy.linalg
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get('num_threads', 1) for i in threadpool_info()
                       if i.get('user_api') == 'blas'] or [os.cpu_count()])
    except Exception:
        threads = os.cpu_count()
    K = matern.dense_correlation(points, 0.1, nu)
    eta = float(etas[0])
    n = K.shape[0]
    t0 = time.perf_counter()
    Kn = K.copy()
    Kn[numpy.diag_indices(n)] += eta
    Y = scipy.linalg.solve(Kn, X, assume_a='pos')          # solve(eta, X)  :62
    Kn = K.copy()
    Kn[numpy.diag_indices(n)] += eta
    w = scipy.linalg.solve(Kn, z, assume_a='pos')          # solve(eta, z)  :332
    _ = (X.T @ Y, w)
    dt = time.perf_counter() - t0
    cpu = platform.processor() or platform.machine()
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    cpu = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    return {'value': 1.0 / dt, 'unit': 'evals/s', 'cores': int(threads), 'kind': 'port',
            'sample': 'one direct log-likelihood eval at N=%d (2 x scipy.linalg.solve '
                      'assume_a=pos, eigen-logdet setup excluded), %.1f s; host %s, '
                      'os.cpu_count()=%d' % (n, dt, cpu, os.cpu_count())}


SPARSE_CONFIGS = {
    # name: (points per axis, dimension, rho, nu, density, probes, lanczos steps, etas)
    'sparse4': (256, 2, 0.005, 1.5, 1e-3, 20, 30, 32),
    'sparse5': (64, 3, 0.02, 1.5, 6e-4, 20, 30, 32),
}


def run_sparse(args, world, rank, local, dist, torch):
    """BASELINE configs 4 / 5: tapered Matern in CSR on the device; per step the
    rank runs the Lanczos of its probe shard (SLQ logdet / traceinv for the
    whole eta grid, one all-gather of per-probe quadratures) and the blocked-CG
    solves of [X | z] for its eta shard (direct lp), then one all-gather of the
    [eta, logdet, lp] rows. The global problem is fixed: scaling "strong"."""
    from gaussian_proc import generate_correlation, _data
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms
    from gaussian_proc.sweep import slq_sweep, shard
    npts, dim, rho, nu, dens, nprobe, steps, neta = SPARSE_CONFIGS[args.config]
    points = _data.generate_points(npts, dim, True)
    z = _data.generate_data(points, 0.2)
    X = _data.generate_basis_functions(points, 2)
    n, m = X.shape
    t_asm = time.perf_counter()
    D = generate_correlation(points, rho, nu, sparse=True, density=dens, device=local,
                             device_resident=True)
    t_asm = time.perf_counter() - t_asm
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': nprobe, 'lanczos_degree': steps})
    # eta grid above |lambda_min| (the tapered matrix is indefinite): smallest Ritz
    # value over the probes of a pilot Lanczos
    a, b = op.sop.lanczos(4, steps, 99)
    from gaussian_proc import _slq
    theta_min = min(float(t.min()) for t, _ in _slq.nodes(a, b))
    shift = max(0.0, -1.1 * theta_min)
    etas = numpy.logspace(-2, 2, neta) + shift
    R = numpy.column_stack([X, z])
    lo, hi, per = shard(neta, world, rank)

    def step():
        curves = slq_sweep(op, etas)
        rows = numpy.zeros((per, 3))
        if hi > lo:
            # all Gram blocks of the eta shard from one multi-shift CG (rtol 1e-6)
            Gs = op.sop.msgram(etas[lo:hi], R, rtol=1e-6)
            for i, e in enumerate(etas[lo:hi]):
                rows[i] = [e, curves['logdet'][lo + i],
                           _lp_from_terms(n, m, 1.0, curves['logdet'][lo + i], Gs[i])]
        t = torch.from_numpy(rows).cuda()
        if world > 1:
            out = torch.empty((world * per, 3), dtype=torch.float64, device=t.device)
            dist.all_gather_into_tensor(out, t)
            return out
        return t

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t_max = torch.tensor([dt], dtype=torch.float64, device='cuda')
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    dt = float(t_max.item())
    # SpMM roofline on a device-resident probe block (HIP events)
    s_blk = max(1, min(32, nprobe // world))
    ms = op.sop.bench_spmm(s_blk, 50)
    nnz = op.sop.nnz
    alg_bytes = 12.0 * nnz + 8.0 * (n + 1) + 16.0 * n * s_blk
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    sp_traffic, sp_tsrc = pmc_traffic_sparse(args.config) if s_blk == 20 else (None, None)
    if rank == 0:
        res = {
            'metric': 'log-likelihood evals/sec (%s, sparse tapered Matern, SLQ + CG)'
                      % args.config,
            'value': neta * args.steps / dt, 'unit': 'evals/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True,
            'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic (reference data_utilities grid, sin + 0.2 noise seed 31)',
            'config': {'workload': '%s: N=%d %dD grid, nu=%g rho=%g density=%g, %d probes x '
                                   '%d Lanczos steps, %d etas' % (args.config, n, dim, nu, rho,
                                                                 dens, nprobe, steps, neta),
                       'n': n, 'nnz': nnz, 'nnz_per_row': nnz / float(n), 'tau': D.tau,
                       'lambda_min_ritz': theta_min, 'eta_shift': shift,
                       'assembly_s': t_asm,
                       'parallelism': 'probe + eta shards x%d + all-gather' % world},
            'roofline': {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(gbs / HBM_PEAK_GBS, 4),
                         'traffic': None if sp_traffic is None else round(sp_traffic),
                         'traffic_unit': 'bytes per launch (HBM side, PMC)',
                         'traffic_source': sp_tsrc,
                         'kernel': 'csr_spmm_kernel (s=%d columns)' % s_blk,
                         'avg_launch_ms': round(ms, 4),
                         # every nonzero gathers s contiguous doubles of X: cache-side bytes
                         'gather_bytes': 8.0 * nnz * s_blk,
                         'gather_gbs': round(8.0 * nnz * s_blk / (ms * 1e-3) / 1e9, 1),
                         'note': 'working set %.1f MB: Infinity-Cache resident when < 256 MB; '
                                 'the X gathers (gather_bytes) are served by L2 / MALL'
                                 % (alg_bytes / 1e6)},
            'lp_sample': [float(v) for v in last[0].tolist()],
            'cpu_baseline': None,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def golden_logdet_err(op_logdet_fn, nu, n):
    """max relative error of logdet(K + eta I) vs the reference's own values
    (tests/golden/cfg3_big.json: eigh/Cholesky of the reference at N=16384,
    nu=1.5, etas 0.01, 1, 4); None for other configurations."""
    path = os.path.join(REPO, 'tests', 'golden', 'cfg3_big.json')
    if n != 16384 or nu != 1.5 or not os.path.isfile(path):
        return None
    with open(path) as fh:
        cfg = json.load(fh)
    ld = numpy.asarray(op_logdet_fn(cfg['etas']))
    ref = numpy.asarray(cfg['logdet'])
    return float(numpy.max(numpy.abs(ld - ref) / numpy.abs(ref)))


def band_mode(args, D, X, z, world, rank, dist, torch, ld_ref=None):
    """The eigenvalue operator's path (MixedCorrelation imate_method='eigenvalue'):
    per step ONE device band reduction K = Q B Q^T of the resident K (redone every
    step), Q^T [X z], and the banded-Cholesky terms of ``--band-etas`` eta values,
    then the host lp and one all-gather. Same eta grid and lp as the dense line."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms
    n, m = X.shape
    E = args.band_etas
    grid = numpy.logspace(-3, 3, max(64, world * E))
    op = MixedCorrelation(D, imate_method='eigenvalue')
    b = op.band()
    acc = {'reduce_ms': 0.0, 'rhs_ms': 0.0, 'loglik_ms': 0.0}

    def step(s, record):
        idx = [(s * world * E + rank * E + j) % grid.size for j in range(E)]
        etas = grid[idx]
        op.refresh_band(X, z)   # reduction of K with Q^T [X z] applied alongside
        ld, G = op.loglik_terms(etas, X, z)
        if record:
            for k, v in b.last_timing().items():
                acc[k] += v
        lp = numpy.array([_lp_from_terms(n, m, 1.0, l, g) for l, g in zip(ld, G)])
        res = torch.from_numpy(numpy.stack([etas, ld, lp], axis=1)).cuda()
        if world > 1:
            out = torch.empty((world * E, 3), dtype=torch.float64, device=res.device)
            dist.all_gather_into_tensor(out, res)
            return out
        return res

    for s in range(args.warmup):
        step(s, False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        last = step(args.warmup + s, True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t_max = torch.tensor([dt], dtype=torch.float64, device='cuda')
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    dt = float(t_max.item())
    K = args.steps
    red = acc['reduce_ms'] / K
    flops_red = 4.0 * n ** 3 / 3.0
    out = {
        'value': world * E * K / dt, 'unit': 'evals/s', 'ms_per_step': dt / K * 1e3,
        'eta_per_rank_per_step': E,
        'step': 'band reduction of K (Q^T [X z] applied alongside) + %d banded Cholesky evals + '
                'host lp' % E,
        'reduce_ms': round(red, 3), 'rhs_ms': round(acc['rhs_ms'] / K, 3),
        'loglik_ms': round(acc['loglik_ms'] / K, 3),
        'marginal_evals_per_s_per_gpu': round(E / (acc['loglik_ms'] / K * 1e-3), 1),
        'reduction_tflops': round(flops_red / (red * 1e-3) / 1e12, 3),
        'reduction_mfma_frac': round(flops_red / (red * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
        'lp_sample': [float(v) for v in last[0].tolist()],
        'logdet_rel_err_vs_reference': golden_logdet_err(
            lambda e: op.loglik_terms(e, X, z)[0], args.nu, n),
    }
    if ld_ref is not None:
        out['logdet_rel_err_vs_cholesky'] = float(numpy.max(
            numpy.abs(op.loglik_terms(ld_ref[0], X, z)[0] - ld_ref[1]) / numpy.abs(ld_ref[1])))
    if not args.no_der:
        out['der1_sweep'] = der1_sweep(op, X, z, E, rank, torch)
    return out


def der1_sweep(op, X, z, E, rank, torch):
    """ProfileLikelihood.log_likelihood_der1_eta over this rank's E points of
    the grid in one call (band Gram blocks G1..G3 + eigenvalue traceinv), after
    the one-time eigenvalues of K (timed separately)."""
    from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood
    log_etas = numpy.linspace(-3, 3, 64)[[(rank * E + j) % 64 for j in range(E)]]
    t0 = time.perf_counter()
    op.eigenvalues()
    eig_ms = (time.perf_counter() - t0) * 1e3
    ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, op, log_etas)   # warm (buffers)
    op._der_cache = None   # time the device work, not the operator's last-call cache
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d1 = ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, op, log_etas)
    dt = time.perf_counter() - t0
    return {'etas': E, 'wall_ms': round(dt * 1e3, 3), 'device_ms': round(op.band().der_ms(), 3),
            'der1_evals_per_s_per_gpu': round(E / dt, 1),
            'eigenvalues_ms_once': round(eig_ms, 1),
            'der1_sample': [float(log_etas[0]), float(d1[0])]}


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    if args.config != 'dense':
        return run_sparse(args, world, rank, local, dist, torch)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    from gaussian_proc import generate_correlation, _data
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms

    points = _data.generate_points(args.grid, 2, True)
    z = _data.generate_data(points, 0.2)
    X = _data.generate_basis_functions(points, 2)
    n, m = X.shape
    B = args.eta_per_rank
    D = generate_correlation(points, 0.1, args.nu, device_resident=True, device=local,
                             max_batch=B)
    op = MixedCorrelation(D)
    op.op.set_outer(args.outer)
    op.op.set_lookahead(args.lookahead)
    op.set_rhs(X, z)
    # 64-point eta grid (cfg3); with more evaluations per step than points over all
    # ranks, a finer grid over the same range, so every rank's eta values are distinct
    grid = numpy.logspace(-3, 3, max(64, world * B))

    def step_etas(s):
        idx = [(s * world * B + rank * B + j) % grid.size for j in range(B)]
        return grid[idx]

    def step(s, timing_acc=None):
        etas = step_etas(s)
        ld, G = op.loglik_terms(etas, X, z)
        if timing_acc is not None:
            t = op.op.last_timing()
            timing_acc['syrk_ms'] += t['syrk_ms']
            timing_acc['syrk_busy_ms'] += t['syrk_busy_ms']
            timing_acc['syrk_flops'] += t['syrk_flops']
            timing_acc['syrk_launches'] += t['syrk_launches']
            timing_acc['total_ms'] += t['total_ms']
        lp = numpy.array([_lp_from_terms(n, m, 1.0, l, g) for l, g in zip(ld, G)])
        res = torch.from_numpy(numpy.stack([etas, ld, lp], axis=1)).cuda()
        if world > 1:
            out = torch.empty((world * B, 3), dtype=torch.float64, device=res.device)
            dist.all_gather_into_tensor(out, res)
            return out
        return res

    for s in range(args.warmup):
        step(s)
    timing = {'syrk_ms': 0.0, 'syrk_busy_ms': 0.0, 'syrk_flops': 0.0, 'syrk_launches': 0,
              'total_ms': 0.0}
    op.op.set_timing(not args.no_timing)
    barrier()
    t0 = time.perf_counter()
    last = None
    for s in range(args.steps):
        last = step(args.warmup + s, None if args.no_timing else timing)
    barrier()
    dt = time.perf_counter() - t0
    op.op.set_timing(False)
    t_max = torch.tensor([dt], dtype=torch.float64, device='cuda')
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    dt = float(t_max.item())
    evals = world * B * args.steps
    flops_eval = n ** 3 / 3.0 + 2.0 * n ** 2 * (m + 1) + n ** 2
    result = None
    if rank == 0:
        roof = None
        if not args.no_timing and timing['syrk_ms'] > 0:
            # algorithmic flops per launch / average launch duration (HIP events on
            # the launching stream) = total flops / summed launch time; with
            # --lookahead 1 launches on the two streams can overlap and busy_ms
            # (their union) is the shorter wall time
            achieved = timing['syrk_flops'] / (timing['syrk_ms'] * 1e-3) / 1e12
            traffic, tsrc = pmc_traffic(args.outer, B)
            roof = {'bound': 'mfma', 'achieved': round(achieved, 3),
                    'peak': FP64_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                    'frac': round(achieved / FP64_MFMA_PEAK_TFLOPS, 4),
                    'traffic': None if traffic is None else round(traffic),
                    'traffic_unit': 'bytes per launch (HBM side, PMC)',
                    'traffic_source': tsrc,
                    'algorithmic_flops_per_launch': round(timing['syrk_flops']
                                                          / max(1, timing['syrk_launches'])),
                    'kernel': 'syrk_kernel (trailing update, fp64 MFMA 16x16x4)',
                    'launches': timing['syrk_launches'],
                    'avg_launch_ms': round(timing['syrk_ms'] / max(1, timing['syrk_launches']), 4),
                    'busy_ms': round(timing['syrk_busy_ms'], 3),
                    'per_launch_tflops': round(timing['syrk_flops'] / (timing['syrk_ms'] * 1e-3)
                                               / 1e12, 3)}
        whole = flops_eval * evals / world / dt / 1e12
        result = {
            'metric': 'log-likelihood evals/sec (N=16384 dense Matern-3/2)',
            'value': evals / dt,
            'unit': 'evals/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': dt / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic (reference data_utilities: 2D grid, sin + 0.2 noise seed 31, '
                    'deg-2 basis)',
            'config': {'workload': 'cfg3: N=%d 2D grid Matern nu=%g rho=0.1, eta grid '
                                   'logspace(-3,3,%d), %d eta/rank/step' % (n, args.nu,
                                                                          grid.size, B),
                       'n': n, 'm': m, 'eta_per_rank_per_step': B,
                       'outer_panel': 128 * args.outer, 'lookahead': args.lookahead,
                       'parallelism': 'eta-shard x%d + all-gather' % world},
            'roofline': roof,
            'whole_eval_tflops_per_gpu': round(whole, 3),
            'whole_eval_mfma_frac': round(whole / FP64_MFMA_PEAK_TFLOPS, 4),
            'flops_per_eval': flops_eval,
            'lp_sample': [float(v) for v in last[0].tolist()] if last is not None else None,
            'cpu_baseline': None,
        }
    ld_err = golden_logdet_err(lambda e: op.loglik_terms(e, X, z)[0], args.nu, n)
    if rank == 0:
        result['logdet_rel_err_vs_reference'] = ld_err
    if not args.no_band:
        ld_ref = (last[:, 0].cpu().numpy()[:B], last[:, 1].cpu().numpy()[:B])
        bm = band_mode(args, D, X, z, world, rank, dist, torch, ld_ref)
        if rank == 0:
            result['band_mode'] = bm
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline(points, z, X, args.nu, step_etas(0))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
