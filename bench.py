#!/usr/bin/env python
"""Benchmark: log-likelihood evaluations / s on the N=16384 dense Matérn-3/2
covariance (BASELINE.json metric), one process per GPU.

A step = the cfg3 eta curve logspace(-3, 3, 64) (``--eta-total``), sharded over
the ranks in contiguous blocks (64 / N eta per rank; strong scaling, BASELINE
cfg3: "64-point eta sweep sharded over 8 x MI355X"): one batched device call per
rank factorizes K + eta_b I (fp64 MFMA Cholesky, fused forward solve of [X | z],
logdet and Gram), the host forms the direct log-likelihood (sigma = 1,
sigma0 = sqrt(eta)), and ONE all-gather (RCCL over xGMI at N > 1) collects the
[eta, logdet, lp] curve. K is assembled on each GPU from the points before the
timed region (inputs resident in HBM). ``--scaling weak`` instead gives every
rank ``--eta-per-rank`` eta of a finer grid (fixed per-rank work).

Launch: python bench.py [--gpus 1 --steps K --warmup W]
        python bench.py --gpus N ...      (starts the N ranks itself: launch_ranks)
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
The world size must equal --gpus; each rank uses device LOCAL_RANK and the line
lists them (``devices``). At N > 1 the line holds the dense curve, the band mode
and the sparse configs 4 and 5 (probe and right-hand-side column shards).
"""

import argparse
import json
import re
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
    ap.add_argument('--scaling', default='strong', choices=['strong', 'weak'],
                    help='strong: the --eta-total point curve split over the ranks (cfg3); '
                         'weak: --eta-per-rank eta per rank of a finer grid')
    ap.add_argument('--eta-total', type=int, default=64,
                    help='strong scaling: eta values of the curve (cfg3: 64)')
    ap.add_argument('--eta-per-rank', type=int, default=64,
                    help='weak scaling: eta values factorized together per rank and step')
    ap.add_argument('--cpu-samples', type=int, default=3,
                    help='CPU baseline: timed evaluations per variant (after one warm-up)')
    ap.add_argument('--cpu-budget-s', type=float, default=20.0,
                    help='sparse CPU baseline: seconds of sampled CG work (extrapolated)')
    ap.add_argument('--outer', type=int, default=16, help='outer panel width / 128')
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
    ap.add_argument('--out-json', default=None,
                    help='also write the JSON line (rank 0) to this file')
    ap.add_argument('--launch-check', action='store_true',
                    help='check the N-rank launch only (no device): world size against '
                         '--gpus, the eta blocks and the all-gather / max-time collectives '
                         'over gloo; prints one JSON line')
    ap.add_argument('--no-extras', action='store_true',
                    help='dense probe runs: skip the batch-efficiency, dense-slq and nu=2.5 '
                         'sub-lines')
    ap.add_argument('--no-sparse', action='store_true',
                    help='dense run: skip the sparse_modes block (configs 4 and 5, N=1 only)')
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
        kernels = json.load(fh)['kernels']
    # template instances appear as 'void gpmi::name<20>'
    k = kernels.get(kernel) or next((v for key, v in kernels.items()
                                     if key.replace('void ', '').split('<')[0] == kernel), None)
    if not k:
        return None, None
    # per_dispatch_first: only the timed call's launches (the run's later
    # golden-logdet call is a smaller batch)
    pd = k.get('per_dispatch_first', k['per_dispatch'])
    return (2.0 * pd['FETCH_SIZE'] + pd['WRITE_SIZE']) * 1024.0, os.path.relpath(files[-1], REPO)


def pmc_traffic_sparse(config, kernel='gpmi::csr_spmm_kernel', width=None):
    """HBM-side bytes per SpMM launch of `kernel` (at block width `width`: template
    instances appear as 'void gpmi::name<12, 8, 4>') from the newest committed PMC
    summary of this sparse config that holds it (profiles/r*/pmc_traffic_{config}.json,
    FETCH_SIZE / WRITE_SIZE passes over `bench.py --config <config> --steps 1`;
    FETCH_SIZE doubled as in pmc_traffic). Per launch: 'per_dispatch_timed' where the
    summary has it (the dispatches of the timed step, between its timing marks),
    else 'per_dispatch_last' (the last K dispatches), else the mean over every
    dispatch of that instance."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*',
                                          'pmc_traffic_%s.json' % config)),
                   key=lambda f: (int(re.search(r'profiles/r(\d+)', f).group(1)), f))
    for f in reversed(files):
        with open(f) as fh:
            kernels = json.load(fh)['kernels']

        def match(key):
            base = key.replace('void ', '')
            if base.split('<')[0] != kernel:
                return False
            return width is None or base.startswith('%s<%d,' % (kernel, width)) or \
                base == '%s<%d>' % (kernel, width)
        k = next((v for key, v in kernels.items() if match(key)), None)
        if not k:
            continue
        pd = k.get('per_dispatch_timed', k.get('per_dispatch_last', k['per_dispatch']))
        return (2.0 * pd['FETCH_SIZE'] + pd['WRITE_SIZE']) * 1024.0, os.path.relpath(f, REPO)
    return None, None


def curve_sha(rows):
    """SHA-256 of the gathered [eta, logdet, lp] rows (float64, C order): equal digests
    at N = 1 and N > 1 mean the curves agree bit for bit."""
    import hashlib
    return hashlib.sha256(numpy.ascontiguousarray(numpy.asarray(rows, dtype=numpy.float64))
                          .tobytes()).hexdigest()


def host_info():
    """The host the CPU baseline runs on: model, logical CPUs, physical cores,
    and the CPUs this job may use (affinity, cgroup quota, OMP_NUM_THREADS: the
    GPU box gives one GPU's job a share of the machine, 16 CPUs)."""
    info = {'logical_cpus': os.cpu_count(), 'cpu_model': platform.processor() or
            platform.machine()}
    phys = set()
    try:
        with open('/proc/cpuinfo') as fh:
            pid = cid = None
            for line in fh:
                if line.startswith('model name'):
                    info['cpu_model'] = line.split(':', 1)[1].strip()
                elif line.startswith('physical id'):
                    pid = line.split(':', 1)[1].strip()
                elif line.startswith('core id'):
                    cid = line.split(':', 1)[1].strip()
                elif not line.strip() and cid is not None:
                    phys.add((pid, cid))
                    pid = cid = None
    except OSError:
        pass
    info['physical_cores'] = len(phys) or None
    try:
        info['affinity_cpus'] = len(os.sched_getaffinity(0))
    except AttributeError:
        info['affinity_cpus'] = os.cpu_count()
    quota = None
    for path in ('/sys/fs/cgroup/cpu.max', '/sys/fs/cgroup/cpu/cpu.cfs_quota_us'):
        try:
            with open(path) as fh:
                parts = fh.read().split()
            if path.endswith('cpu.max') and parts[0] != 'max':
                quota = int(parts[0]) / float(parts[1])
            elif path.endswith('quota_us') and int(parts[0]) > 0:
                with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as fh:
                    quota = int(parts[0]) / float(fh.read().split()[0])
            break
        except (OSError, ValueError, IndexError):
            continue
    info['cgroup_cpu_quota'] = quota
    usable = info['affinity_cpus']
    if quota:
        usable = min(usable, max(1, int(quota)))
    omp = os.environ.get('OMP_NUM_THREADS')
    if omp and omp.isdigit() and int(omp) > 0:
        usable = min(usable, int(omp))
    info['job_cpus'] = usable
    return info


def log(msg):
    """Progress on stderr (the JSON result is the only stdout line)."""
    sys.stderr.write('[bench] %s\n' % msg)
    sys.stderr.flush()


def emit(args, line):
    """The ONE stdout JSON line (rank 0); with --out-json also into that file."""
    txt = json.dumps(line)
    print(txt, flush=True)
    if getattr(args, 'out_json', None):
        with open(args.out_json, 'w') as fh:
            fh.write(txt + '\n')


def _timed(fn, reps, what=None):
    out = []
    for r in range(reps):
        t0 = time.perf_counter()
        v = fn()
        out.append((time.perf_counter() - t0, v))
        if what:
            log('%s %d/%d: %.2f s' % (what, r + 1, reps, out[-1][0]))
    return out


def cpu_baseline(points, z, X, nu, eta, lam=None, samples=3):
    """The reference's CPU call pattern, timed on this host (rank 0, N=1), by
    the oracle restatement (kind 'port'; the reference itself never travels):
    DirectLikelihood.log_likelihood (_direct_likelihood.py:31-83) at
    (sigma, sigma0) = (1, sqrt(eta)) on
      * the 'eigenvalue' operator Likelihood builds (likelihood.py:41):
        O(n) eigen-logdet + 2 x scipy.linalg.solve(K + eta I, ., assume_a='pos')
        (mixed_correlation.py:239-248,280-299); the one-time eigh(K) setup
        (:76-79; 227 s at this N on 8 cores) is excluded. Its eigenvalues are
        the device's (lam) when given, so the CPU lp is comparable;
      * the 'cholesky' variant: a third factorization for logdet (:250-261).
    BLAS threads = every CPU this job may use (host_info); one warm-up eval,
    then the median of ``samples`` evals per variant."""
    from oracle import matern
    from oracle import likelihood as olk
    from oracle.mixed_correlation import MixedCorrelation as OracleMC
    from threadpoolctl import threadpool_limits, threadpool_info
    info = host_info()
    threads = info['job_cpus']
    log('cpu baseline: host %s, %d job CPUs; assembling K' % (info['cpu_model'], threads))
    K = matern.dense_correlation(points, 0.1, nu)
    n = K.shape[0]
    hp = [1.0, float(numpy.sqrt(eta))]
    with threadpool_limits(limits=threads, user_api='blas'):
        blas = [(i.get('internal_api'), i.get('num_threads')) for i in threadpool_info()
                if i.get('user_api') == 'blas']
        eig = OracleMC(K, 'cholesky')
        eig.imate_method = 'eigenvalue'
        eig.K_eigenvalues = numpy.asarray(lam, dtype=float) if lam is not None else numpy.ones(n)
        chol = OracleMC(K, 'cholesky')
        warm = _timed(lambda: olk.direct_lp(z, X, eig, hp), 1, 'cpu warm-up eval')
        te = _timed(lambda: olk.direct_lp(z, X, eig, hp), samples, 'cpu eigenvalue-operator eval')
        tc = _timed(lambda: olk.direct_lp(z, X, chol, hp), samples, 'cpu cholesky-variant eval')
    med_e = float(numpy.median([t for t, _ in te]))
    med_c = float(numpy.median([t for t, _ in tc]))
    out = {'value': 1.0 / med_e, 'unit': 'evals/s', 'cores': int(threads), 'kind': 'port',
           'sample': 'DirectLikelihood.log_likelihood at N=%d, eta=%g: median of %d evals after '
                     '1 warm-up, eigenvalue operator (eigen-logdet + 2 x '
                     'scipy.linalg.solve(assume_a=pos); one-time eigh excluded), BLAS threads=%d'
                     % (n, eta, samples, threads),
           'median_s': round(med_e, 3), 'samples_s': [round(t, 3) for t, _ in te],
           'warmup_s': round(warm[0][0], 3),
           'cholesky_variant': {'value': 1.0 / med_c, 'unit': 'evals/s', 'median_s':
                                round(med_c, 3), 'samples_s': [round(t, 3) for t, _ in tc],
                                'step': '3 factorizations per eval (logdet + 2 solves)'},
           'threads': int(threads), 'blas': blas, 'host': info}
    if info.get('physical_cores'):
        # what every physical core of the host could do at perfect BLAS scaling
        # (an upper bound for the CPU; the box gives this job job_cpus of them)
        out['all_physical_cores_upper_bound'] = {
            'cores': info['physical_cores'],
            'value': out['value'] * info['physical_cores'] / float(threads),
            'note': 'linear extrapolation from %d to %d cores (optimistic for the CPU)'
                    % (threads, info['physical_cores'])}
    if lam is not None:
        out['lp_eigen'] = float(te[0][1])
    out['lp_cholesky'] = float(tc[0][1])
    return out


def cpu_baseline_sparse(K, X, z, etas, nprobe, steps, seed, budget_s, workers=None,
                        reorth=False):
    """Restated reference pattern for a sparse K on scipy (the shipped sparse
    path cannot run: SURVEY 0.4): stochastic Lanczos quadrature with the SAME
    counter-based probes and the same recurrence as the device (oracle.sparse: CSR
    SpMV Lanczos, plain three-term for imate's orthogonalize = 0, else CGS2)
    for logdet at every eta, and per eta the reference's solves of X and z
    column by column with scipy.sparse.linalg.cg, rtol 1e-6
    (_linear_solver.py:57-68). The probes and the (eta, column) solves are
    independent, so they run on a thread pool over every CPU this job may use
    (host_info; scipy's CSR SpMV and numpy's vector kernels release the GIL,
    BLAS pinned to one thread per worker). Bounded sample: all probes' Lanczos,
    then CG solves of spread eta until ``budget_s`` of wall time is spent,
    extrapolated to the whole grid at the measured pool throughput."""
    import scipy.sparse
    import scipy.sparse.linalg
    from concurrent.futures import ThreadPoolExecutor
    from threadpoolctl import threadpool_limits
    from oracle import sparse as osp
    n = K.shape[0]
    info = host_info()
    workers = int(workers or info['job_cpus'])
    K = K.tocsr()
    P = osp.rademacher_probes(n, nprobe, seed)
    R = numpy.column_stack([X, z])
    eye = scipy.sparse.identity(n, format='csr')
    # (eta, column) tasks with the etas spread over the grid
    order = numpy.argsort(numpy.arange(etas.size) % 4, kind='stable')
    tasks = [(j, c) for j in order for c in range(R.shape[1])]
    mats = {}

    def lanczos(p):
        return osp.lanczos(K, P[:, p], steps, reorth=reorth)

    def solve(task):
        j, c = task
        cnt = [0]
        x, _ = scipy.sparse.linalg.cg(mats[j], R[:, c], rtol=1e-6, atol=0.0,
                                      callback=lambda xk: cnt.__setitem__(0, cnt[0] + 1))
        # the Gram column R^T x (checked against the device's multi-shift CG)
        return cnt[0], (j, c, R.T @ x)
    with threadpool_limits(limits=1, user_api='blas'), ThreadPoolExecutor(workers) as ex:
        t0 = time.perf_counter()
        ab = list(ex.map(lanczos, range(nprobe)))
        t_slq = time.perf_counter() - t0
        log('cpu SLQ (%d probes, %d threads): %.1f s' % (nprobe, workers, t_slq))
        for j in order:
            mats[j] = (K + etas[j] * eye).tocsr()
        t0 = time.perf_counter()
        futs, its, k = [], [], 0
        # keep the pool full; stop issuing once the budget is spent
        while k < len(tasks) and (k < workers or time.perf_counter() - t0 < budget_s):
            futs.append(ex.submit(solve, tasks[k]))
            k += 1
            if len(futs) >= workers:
                its.append(futs.pop(0).result())
        its += [f.result() for f in futs]
        t_cg = time.perf_counter() - t0
    cols = [g for _, g in its]
    its = [i for i, _ in its]
    done = len(its)
    log('cpu CG: %d solves in %.1f s on %d threads' % (done, t_cg, workers))
    total = t_slq + t_cg * (etas.size * R.shape[1]) / float(done)
    theta = [osp.slq_nodes(a, b) for a, b in ab]
    logdet = numpy.array([n * numpy.mean([numpy.sum(w * numpy.log(t + e)) for t, w in theta])
                          for e in etas])
    return {'value': etas.size / total, 'unit': 'evals/s', 'cores': workers, 'kind': 'port',
            'sample': 'SLQ of all %d probes x %d Lanczos steps (%.1f s, same probes as the '
                      'device) + %d of %d CG solves (rtol 1e-6, %.1f s, mean %.0f iterations), '
                      'on a %d-thread pool, extrapolated to the %d-eta grid'
                      % (nprobe, steps, t_slq, done, etas.size * R.shape[1], t_cg,
                         numpy.mean(its), workers, etas.size),
            'slq_s': round(t_slq, 3), 'cg_s_per_solve_wall': round(t_cg / done, 4),
            'est_s_per_step': round(total, 2), 'threads': workers, 'host': info,
            'logdet': logdet.tolist(), 'gram_columns': cols}


def sparse_step_bytes(n, nnz, s_lanczos, steps, s_cg, cg_iters, orthogonalize=0,
                      cg_segments=None):
    """Algorithmic bytes of one sparse step as implemented (each vector block
    read or written once per pass). Lanczos (block b_L = 8 n s_L): with
    orthogonalize = 0 (imate's default, the plain recurrence, gpmi_sparse.hip
    lz0_*) per step the SpMM (12 nnz + 8(n+1) + 2 b_L, u . Ku in its epilogue) and
    the update pass (y, u_{k-1}, u_k read, u_{k+1} written: 4 b_L); with -1, DCGS2
    (lz_*): per step k the SpMM, the dot pass over the k basis blocks, u and y
    ((k + 2) b_L) and the update pass (k basis blocks, u, y read; v_k, u written:
    (k + 4) b_L), then one final dot pass over the basis and u ((steps + 1) b_L).
    Multi-shift CG (b_C = 8 n s_C, s_C the device width: a full 11-column block on
    the window SpMM is padded by one zero column) per iteration: the SpMM (p . q in
    its epilogue), the r update with B^T r / r . r on MFMA (b, r, q read, r
    written: 4 b_C) and p = r + beta p (3 b_C). cg_segments: the CG's launch
    segments [(device width, iterations), ...] (gpmi_sp_msgram_segments: the full
    block, then the block its active-column compaction narrowed it to); without
    them cg_iters iterations at width s_cg."""
    csr = 12.0 * nnz + 8.0 * (n + 1)
    bl, bc = 8.0 * n * s_lanczos, 8.0 * n * s_cg
    if orthogonalize == 0:
        lanczos = steps * (csr + 2 * bl + 4 * bl)
        basis = 0.0
    else:
        lanczos = sum(csr + 2 * bl + (k + 2) * bl + (k + 4) * bl for k in range(steps)) + \
            (steps + 1) * bl
        basis = sum(2.0 * k * bl for k in range(steps)) + steps * bl
    if cg_segments is None:
        cg_segments = [(s_cg, cg_iters)]
    cg = sum(k * (csr + 9 * 8.0 * n * w) for w, k in cg_segments)
    return {'lanczos': lanczos, 'lanczos_basis_reads': basis, 'cg': cg,
            'total': lanczos + cg}


SPARSE_CONFIGS = {
    # name: (points per axis, dimension, rho, nu, density, probes, lanczos steps, etas)
    'sparse4': (256, 2, 0.005, 1.5, 1e-3, 20, 30, 32),
    'sparse5': (64, 3, 0.02, 1.5, 6e-4, 20, 30, 32),
}


def run_sparse(args, world, rank, local, dist, torch, devices=None):
    """``--config sparse4|sparse5``: the sparse line alone (sparse_measure)."""
    res = sparse_measure(args, args.config, world, rank, local, dist, torch,
                         cpu=world == 1 and not args.no_cpu_baseline, exact=True)
    if rank == 0:
        res['devices'] = devices
        emit(args, res)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def sparse_measure(args, config, world, rank, local, dist, torch, cpu, exact, defer_cpu=False):
    """BASELINE configs 4 / 5: tapered Matern in CSR on the device; per step the
    rank runs the Lanczos of its probe shard (SLQ logdet / traceinv for the
    whole eta grid, one all-gather of per-probe quadratures) and the blocked-CG
    solves of [X | z] for its eta shard (direct lp), then one all-gather of the
    [eta, logdet, lp] rows. The global problem is fixed: scaling "strong".
    Returns the line (rank 0; None elsewhere). ``exact``: the reference check
    also runs the exact 'cholesky' method on a dense copy (cfg 4: 34 GB)."""
    from gaussian_proc import generate_correlation, _data
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms_batch
    from gaussian_proc.sweep import slq_gram_sweep, shard
    npts, dim, rho, nu, dens, nprobe, steps, neta = SPARSE_CONFIGS[config]
    points = _data.generate_points(npts, dim, True)
    z = _data.generate_data(points, 0.2)
    X = _data.generate_basis_functions(points, 2)
    n, m = X.shape
    t_asm = time.perf_counter()
    D = generate_correlation(points, rho, nu, sparse=True, density=dens, device=local,
                             device_resident=True)
    t_asm = time.perf_counter() - t_asm
    # imate's defaults otherwise: orthogonalize=0, the plain three-term recurrence
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': nprobe, 'lanczos_degree': steps})
    # eta grid above |lambda_min| (the tapered matrix is indefinite): smallest Ritz
    # value over the SLQ probes' own Lanczos (Ritz values converge to lambda_min
    # from above: 10 % margin; the SLQ shift check and the CG curvature check
    # raise LinAlgError if K + eta I is still not positive definite)
    from gaussian_proc import _slq
    theta_min = _slq.min_ritz(op.slq_nodes())
    shift = max(0.0, -1.1 * theta_min)
    etas = numpy.logspace(-2, 2, neta) + shift
    R = numpy.column_stack([X, z])
    # [X | z] is input data: resident in HBM before the timed region (gpmi_sp_set_rhs),
    # as K is, so a step does not upload it (cfg 5: 23 MB, ~1.9 ms from pageable memory)
    op.sop.set_rhs(R)
    lo, hi, per = shard(neta, world, rank)

    holder = {'cg_iters': 0, 'cg_segments': None}

    def step():
        # the SLQ Lanczos of the probe shard and the multi-shift CG Gram blocks of
        # the eta shard (rtol 1e-6) run together on two streams (sweep.slq_gram_sweep)
        curves, _, Gs = slq_gram_sweep(op, etas, None, rtol=1e-6)
        holder['curves'] = curves
        holder['grams'] = Gs
        rows = numpy.zeros((per, 3))
        if hi > lo:
            holder['cg_iters'] = op.sop.last_cg_iterations
            holder['cg_segments'] = op.sop.msgram_segments()
            ld = curves['logdet'][lo:hi]
            rows[:hi - lo, 0] = etas[lo:hi]
            rows[:hi - lo, 1] = ld
            rows[:hi - lo, 2] = _lp_from_terms_batch(n, m, 1.0, ld, Gs)
        return gather_rows(rows, world, dist, torch)

    for _ in range(args.warmup):
        step()
    # in-step SpMM timing over the timed steps themselves: every window SpMM launch
    # stamps its span (earliest workgroup start to latest workgroup end, the device's
    # constant wall clock, two vector atomics per workgroup) into a slot of its own;
    # the window is marked in a kernel trace by two timing_mark_kernel launches
    op.sop.set_timing(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    op.sop.set_timing(False)
    spmm_in_step = op.sop.spmm_timing()
    dt = max_over_ranks(dt, world, dist, torch)
    # imate's `orthogonalize` option: this rank's probe block by the plain three-term
    # recurrence (0, imate's default, what the step uses) against full
    # reorthogonalisation (-1, DCGS2), Lanczos alone, and the two logdet curves in
    # probe standard errors
    lz = None
    if rank == 0:
        plo, phi, _ = shard(nprobe, world, rank)
        lzt = {}
        curves = {}
        for orth in (-1, 0):
            op.sop.lanczos(phi - plo, steps, op.seed, probe_offset=plo, orthogonalize=orth)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            a_, b_ = op.sop.lanczos(phi - plo, steps, op.seed, probe_offset=plo,
                                    orthogonalize=orth)
            lzt[orth] = (time.perf_counter() - t1) * 1e3
            curves[orth] = n * _slq.quadrature(_slq.nodes(a_, b_), etas, numpy.log)
        se = curves[-1].std(axis=0, ddof=1) / numpy.sqrt(curves[-1].shape[0])
        dz = (curves[0].mean(axis=0) - curves[-1].mean(axis=0)) / se
        lz = {'probes': phi - plo, 'steps': steps, 'full_reorth_ms': round(lzt[-1], 3),
              'orthogonalize_0_ms': round(lzt[0], 3),
              'logdet_diff_in_std_errors_max': round(float(numpy.max(numpy.abs(dz))), 3),
              'note': "the measured step uses imate's default orthogonalize=0 (plain "
                      "three-term recurrence); -1 is full reorthogonalisation (DCGS2)"}
    # SpMM roofline from the timed steps: the multi-shift CG's SpMM (its block width;
    # the step's critical path: the step waits for the CG, which runs at the high
    # dispatch priority, while the Lanczos beside it has slack and its launches' spans
    # stretch around the CG's), else the width with the most device time; its
    # average in-step launch span; the same kernel isolated (50 back-to-back launches
    # on a resident block) is reported beside it as isolated_ms
    nnz = op.sop.nnz
    # the library pads a full 11-column block on the window SpMM to 12 (msgram_impl);
    # a column shard (N > 1) runs unpadded: rank 0's shard width
    clo0, chi0, _ = shard(R.shape[1], world, 0)
    s_cg = (chi0 - clo0) + (1 if (world == 1 and R.shape[1] == 11 and
                                  op.sop.spmm_kernel(11) == 'csr_spmm_wing_kernel') else 0)
    s_blk = (s_cg if s_cg in spmm_in_step
             else max(spmm_in_step, key=lambda w: spmm_in_step[w][1]))
    n_launch, tot_ms = spmm_in_step[s_blk]
    ms_span = tot_ms / n_launch
    # the stamps span a launch's first workgroup start to its last workgroup end; a
    # dispatch also costs the command processor's launch and the end-of-kernel
    # release, which a kernel trace's dispatch interval includes. Measured here on
    # the same kernel: 50 back-to-back launches' period per launch (HIP events
    # around them) less their mean stamped span
    op.sop.set_timing(True)
    ms_iso = op.sop.bench_spmm(s_blk, 50)
    op.sop.set_timing(False)
    iso_n, iso_tot = op.sop.spmm_timing()[s_blk]
    # iso_n: the 50 gated launches only (gpmi_sp_bench_spmm keeps its warm-up out of the log)
    dispatch_ms = max(0.0, ms_iso - iso_tot / iso_n)
    ms = ms_span + dispatch_ms
    alg_bytes = 12.0 * nnz + 8.0 * (n + 1) + 16.0 * n * s_blk
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    info = op.sop.spmm_info()
    sp_kernel = op.sop.spmm_kernel(s_blk)
    windowed = info['windowed'] or sp_kernel == 'csr_spmm_wing_kernel'
    gather_bytes = (8.0 * s_blk * info['mean_window'] * ((n + 63) // 64) if windowed
                    else 8.0 * nnz * s_blk)
    sp_traffic, sp_tsrc = pmc_traffic_sparse(config, 'gpmi::' + sp_kernel, s_blk)
    by_width = {str(w): {'launches': c, 'total_ms': round(t, 3),
                         'avg_launch_ms': round(t / c, 4),
                         'frac': round((12.0 * nnz + 8.0 * (n + 1) + 16.0 * n * w) /
                                       (t / c * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                for w, (c, t) in sorted(spmm_in_step.items())}
    my_probes = shard(nprobe, world, rank)
    sb = sparse_step_bytes(n, nnz, my_probes[1] - my_probes[0], steps, s_cg,
                           holder['cg_iters'], op.orthogonalize, holder['cg_segments'])
    step_s = dt / args.steps
    res = None
    if rank == 0:
        res = {
            'metric': 'log-likelihood evals/sec (%s, sparse tapered Matern, SLQ + CG)'
                      % config,
            'value': neta * args.steps / dt, 'unit': 'evals/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True,
            'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic (reference data_utilities grid, sin + 0.2 noise seed 31)',
            'config': {'workload': '%s: N=%d %dD grid, nu=%g rho=%g density=%g, %d probes x '
                                   '%d Lanczos steps (orthogonalize=%d), %d etas'
                                   % (config, n, dim, nu, rho, dens, nprobe, steps,
                                      op.orthogonalize, neta),
                       'n': n, 'nnz': nnz, 'nnz_per_row': nnz / float(n), 'tau': D.tau,
                       'lambda_min_ritz': theta_min, 'eta_shift': shift,
                       'assembly_s': t_asm,
                       'parallelism': ('probe shards + right-hand-side column shards x%d, '
                                       'all-gathers' % world) if world > 1 else 'one GPU'},
            'roofline': {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(gbs / HBM_PEAK_GBS, 4),
                         'traffic': None if sp_traffic is None else round(sp_traffic),
                         'traffic_unit': 'bytes per launch (HBM side, PMC)',
                         'traffic_source': sp_tsrc,
                         'kernel': '%s (s=%d columns)' % (sp_kernel, s_blk),
                         'avg_launch_ms': round(ms, 4),
                         'avg_launch_ms_source': 'in_step_span_ms (device wall-clock span, '
                                                 'first workgroup start to last workgroup '
                                                 'end, of each SpMM launch of the %d timed '
                                                 'steps: %d launches at s=%d) + '
                                                 'dispatch_overhead_ms' % (args.steps, n_launch,
                                                                           s_blk),
                         'in_step_span_ms': round(ms_span, 5),
                         'dispatch_overhead_ms': round(dispatch_ms, 5),
                         'dispatch_overhead_source': '50 back-to-back launches of the same '
                                                     'kernel: period per launch (HIP events) '
                                                     'less their mean stamped span',
                         'frac_of_span': round(alg_bytes / (ms_span * 1e-3) / 1e9 /
                                               HBM_PEAK_GBS, 4),
                         'isolated_ms': round(ms_iso, 4),
                         'algorithmic_bytes_per_launch': alg_bytes,
                         'in_step_by_width': by_width,
                         # cache-side X bytes: every nonzero gathers s contiguous doubles
                         # (gather kernel), or every 64-row block stages its window
                         'gather_bytes': gather_bytes,
                         'gather_gbs': round(gather_bytes / (ms * 1e-3) / 1e9, 1),
                         'spmm_window': info,
                         'note': 'working set %.1f MB: Infinity-Cache resident when < 256 MB; '
                                 'the X reads (gather_bytes) are served by L2 / MALL'
                                 % (alg_bytes / 1e6)},
            # the whole step against HBM: algorithmic bytes of every pass of the
            # step (sparse_step_bytes) / ms_per_step, rank 0's shard
            'lanczos_orthogonalize': lz,
            'step_roofline': {
                'bound': 'hbm', 'bytes_per_step': sb['total'],
                'achieved': round(sb['total'] / step_s / 1e9, 1), 'peak': HBM_PEAK_GBS,
                'unit': 'GB/s', 'frac': round(sb['total'] / step_s / 1e9 / HBM_PEAK_GBS, 4),
                'lanczos_bytes': sb['lanczos'], 'lanczos_basis_read_bytes':
                    sb['lanczos_basis_reads'], 'cg_bytes': sb['cg'],
                'cg_iterations': holder['cg_iters'],
                # (device width, iterations launched) of the full block and of the
                # block the active-column compaction narrowed it to
                'cg_segments': holder['cg_segments'],
                'lanczos_probes': my_probes[1] - my_probes[0], 'lanczos_steps': steps,
                'cg_columns': R.shape[1], 'cg_device_width': s_cg,
                'lanczos_orthogonalize': op.orthogonalize,
                'model': 'bench.sparse_step_bytes (each vector block once per pass)'},
            'lp_sample': [float(v) for v in last[0].tolist()],
            # every eta of the curve finite (round 6: a large shift's Gram was NaN)
            'lp_all_finite': bool(numpy.all(numpy.isfinite(last[:, 1:]))),
            'curve_sha256': curve_sha(last),
            'cpu_baseline': None,
        }
        ref = sparse_reference_check(op, config, X, z, exact)
        if ref:
            res['reference_check'] = ref
        if cpu:
            csr, seed = op.sop.csr(), op.seed

            def cpu_leg():
                cpu_baseline_leg(res, holder, csr, X, z, etas, nprobe, steps, seed,
                                 args.cpu_budget_s, reorth=op.orthogonalize != 0)
            if defer_cpu:
                # run by the caller after every device measurement (host-side leftovers of
                # the CPU baseline's thread pool slowed the launch-bound sparse steps that
                # followed it: cfg 4 6.2 -> 7.3 ms)
                res['_cpu_leg'] = cpu_leg
            else:
                cpu_leg()
    op.sop.close()
    return res


def cpu_baseline_leg(res, holder, csr, X, z, etas, nprobe, steps, seed, budget_s,
                     reorth=False):
    """The sparse line's CPU baseline (cpu_baseline_sparse) and its checks against the
    device results of the timed steps (holder), into res."""
    cb = cpu_baseline_sparse(csr, X, z, etas, nprobe, steps, seed, budget_s, reorth=reorth)
    dev = holder['curves']['logdet']
    cb['slq_logdet_rel_diff_vs_device_same_probes'] = float(
        numpy.max(numpy.abs(numpy.asarray(cb.pop('logdet')) - dev) / numpy.abs(dev)))
    # the Gram columns the host CG solved (both at rtol 1e-6) against the device's
    # multi-shift CG blocks of the last timed step (rank 0 holds every eta at N=1)
    Gd = holder['grams']
    cb['cg_gram_column_rel_diff_vs_device_max'] = float(max(
        numpy.max(numpy.abs(numpy.asarray(Gd[j])[:, c] - g)) /
        numpy.max(numpy.abs(numpy.asarray(Gd[j])[:, c]))
        for j, c, g in cb.pop('gram_columns')))
    res['cpu_baseline'] = cb
    res['speedup_vs_cpu'] = round(res['value'] / cb['value'], 1)


def sparse_modes(args, world, rank, local, dist, torch):
    """The sparse configs 4 and 5 in the default (dense) line, each with its own
    value, step time, SpMM and whole-step rooflines, reference check and (N=1)
    thread-pool CPU baseline (sparse_measure; the exact-Cholesky leg of the
    reference check is left to --config sparse4). At N > 1 every rank runs its
    probe shard and right-hand-side column shard (BASELINE cfg5: "sharded over
    8 x MI355X with RCCL all-gather"); rank 0 returns the lines, the others None."""
    out, res = {}, {}
    for cfg in ('sparse4', 'sparse5'):
        res[cfg] = sparse_measure(args, cfg, world, rank, local, dist, torch,
                                  cpu=world == 1 and not args.no_cpu_baseline, exact=False,
                                  defer_cpu=True)
        if rank == 0:
            log('%s: %.1f evals/s' % (cfg, res[cfg]['value']))
    if rank != 0:
        return None
    # the CPU baselines after both device measurements
    for cfg in ('sparse4', 'sparse5'):
        leg = res[cfg].pop('_cpu_leg', None)
        if leg:
            leg()
    for cfg in ('sparse4', 'sparse5'):
        r = res[cfg]
        out[cfg] = {k: r[k] for k in ('metric', 'value', 'unit', 'n_gpus', 'ms_per_step',
                                      'steps', 'warmup', 'scaling', 'roofline',
                                      'step_roofline', 'cpu_baseline', 'lp_sample',
                                      'curve_sha256', 'lp_all_finite',
                                      'lanczos_orthogonalize') if k in r}
        out[cfg]['parallelism'] = r['config']['parallelism']
        out[cfg]['workload'] = r['config']['workload']
        out[cfg]['assembly_s'] = r['config']['assembly_s']
        for k in ('reference_check', 'speedup_vs_cpu'):
            if k in r:
                out[cfg][k] = r[k]
    return out


def sparse_reference_check(op, config, X, z, exact=True):
    """BASELINE cfg4 against the reference's own exact values
    (tests/golden/sparse_cfg4.json: reference generator + the 2 argument fixes,
    SuperLU logdet and Gram at three eta above |lambda_min|): the device CSR
    (nnz, sum), the multi-shift CG Gram blocks (rtol 1e-10) and the SLQ logdet
    with its Monte-Carlo standard error over the probes."""
    from gaussian_proc import _slq
    name = {'sparse4': 'sparse_cfg4.json', 'sparse5': 'sparse_cfg5.json'}[config]
    path = os.path.join(REPO, 'tests', 'golden', name)
    if not os.path.isfile(path):
        return None
    with open(path) as fh:
        g = json.load(fh)
    out = {'fixture': name, 'nnz_equal': op.sop.nnz == g['nnz'],
           'data_sum_rel_err': abs(float(op.sop.csr().data.sum()) - g['data_sum']) /
           g['data_sum']}
    if 'etas' in g:
        R = numpy.column_stack([X, z])
        G = op.sop.msgram(g['etas'], R, rtol=1e-10)
        out['gram_rel_err'] = float(max(numpy.max(numpy.abs(Gj - numpy.asarray(Gr))) /
                                        numpy.max(numpy.abs(Gr)) for Gj, Gr in zip(G, g['gram'])))
        q = _slq.quadrature(op.slq_nodes(), g['etas'], _slq.FUNCS['logdet']) * op.n
        est, se = q.mean(axis=0), q.std(axis=0, ddof=1) / numpy.sqrt(q.shape[0])
        out['slq_logdet_err_in_std_errors'] = [round(float(v), 3) for v in
                                               numpy.abs(est - g['logdet']) / se]
        if exact and op.n <= 65536:
            # the exact 'cholesky' method on this sparse K (dense device copy,
            # fp64 MFMA Cholesky per eta) against the same SuperLU values
            from gaussian_proc._mixed_correlation import MixedCorrelation
            ex = MixedCorrelation(op.K, imate_method='cholesky')
            t0 = time.perf_counter()
            ex._dense()
            t_copy = time.perf_counter() - t0
            t0 = time.perf_counter()
            ld, Ge = ex.loglik_terms(g['etas'], X, z)
            t_eval = (time.perf_counter() - t0) / len(g['etas'])
            out['exact_cholesky'] = {
                'dense_copy_s': round(t_copy, 3), 'per_eta_s': round(t_eval, 3),
                'logdet_rel_err': float(numpy.max(numpy.abs(ld - g['logdet']) /
                                                  numpy.abs(g['logdet']))),
                'gram_rel_err': float(max(numpy.max(numpy.abs(Gj - numpy.asarray(Gr))) /
                                          numpy.max(numpy.abs(Gr))
                                          for Gj, Gr in zip(Ge, g['gram'])))}
            ex.op.close()
            del ex
    return out


def golden_case(nu, n):
    """The reference's own N=16384 values for this kernel (tests/golden:
    cfg3_big.json nu=1.5, cfg3_nu25.json nu=2.5; 'cholesky' imate method, made
    by tests/golden/make_golden.py), or None."""
    name = {1.5: 'cfg3_big.json', 2.5: 'cfg3_nu25.json'}.get(nu)
    path = os.path.join(REPO, 'tests', 'golden', name) if name else None
    if n != 16384 or path is None or not os.path.isfile(path):
        return None
    with open(path) as fh:
        return json.load(fh)


def golden_errors(terms_fn, nu, n, m):
    """max relative errors of logdet(K + eta I) at the golden etas and of the
    direct log-likelihood at the golden (sigma, sigma0), vs the reference.
    terms_fn(etas) -> (logdet[], G[]) of the operator under test."""
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms
    cfg = golden_case(nu, n)
    if cfg is None:
        return None, None
    ld = numpy.asarray(terms_fn(cfg['etas'])[0])
    ld_err = float(numpy.max(numpy.abs(ld - cfg['logdet']) / numpy.abs(cfg['logdet'])))
    lp_err = 0.0
    for (sg, s0), ref in zip(cfg['hypers'], cfg['direct_lp']):
        l, G = terms_fn([(s0 / sg) ** 2])
        lp = _lp_from_terms(n, m, sg, l[0], G[0])
        lp_err = max(lp_err, abs(lp - ref) / abs(ref))
    return ld_err, float(lp_err)


def eta_block(args, world, rank, s=0):
    """This rank's eta of step s: strong scaling, the rank's contiguous block of
    the --eta-total curve (gaussian_proc.sweep.shard, padded blocks repeat the
    block's last eta so every rank factorizes the same batch size); weak
    scaling, --eta-per-rank eta of logspace(-3, 3, N * eta_per_rank)."""
    from gaussian_proc.sweep import shard
    if args.scaling == 'strong':
        grid = numpy.logspace(-3, 3, args.eta_total)
        lo, hi, per = shard(grid.size, world, rank)
        idx = list(range(lo, hi)) or [grid.size - 1]
        idx += [idx[-1]] * (per - len(idx))
        return grid[idx], hi - lo, per, grid.size
    B = args.eta_per_rank
    grid = numpy.logspace(-3, 3, max(64, world * B))
    idx = [(s * world * B + rank * B + j) % grid.size for j in range(B)]
    return grid[idx], B, B, grid.size


def max_over_ranks(dt, world, dist, torch):
    """Wall time of the slowest rank (all-reduce MAX; a device tensor on RCCL,
    a host tensor on gloo). ``dist`` None: no process group."""
    if dist is None:
        return dt
    dev = 'cuda' if dist.get_backend() == 'nccl' else 'cpu'
    t_max = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    return float(t_max.item())


def gather_rows(rows, world, dist, torch):
    """ONE all-gather of the per-rank [eta, logdet, lp] rows (RCCL over xGMI for
    the nccl backend, gloo on CPU in the tests): gaussian_proc.sweep's
    collective. Returns the [world * rows, 3] host array on every rank."""
    rows = numpy.ascontiguousarray(rows)
    if dist is None:
        torch.cuda.synchronize()
        return rows
    from gaussian_proc.sweep import _all_gather_rows
    return _all_gather_rows(dist, None, rows, world)


def band_mode(args, D, X, z, world, rank, dist, torch, ld_ref=None):
    """The eigenvalue operator's path (MixedCorrelation imate_method='eigenvalue'):
    per step ONE device band reduction K = Q B Q^T of the resident K (redone every
    step), Q^T [X z], and the banded-Cholesky terms of this rank's eta block, then
    the host lp and one all-gather. Same eta blocks and lp as the dense line.
    The reduction is the operator's one-time setup: every rank repeats it for
    its own K (it does not shard); only the per-eta banded Cholesky does."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms_batch
    n, m = X.shape
    op = MixedCorrelation(D, imate_method='eigenvalue')
    b = op.band()
    acc = {'reduce_ms': 0.0, 'rhs_ms': 0.0, 'loglik_ms': 0.0}

    def step(s, record):
        etas, own, per, _ = eta_block(args, world, rank, s)
        if args.scaling == 'weak':
            etas = etas[:args.band_etas]
        op.refresh_band(X, z)   # reduction of K with Q^T [X z] applied alongside
        ld, G = op.loglik_terms(etas, X, z)
        if record:
            for k, v in b.last_timing().items():
                acc[k] += v
        lp = _lp_from_terms_batch(n, m, 1.0, ld, G)
        return gather_rows(numpy.stack([etas, ld, lp], axis=1), world, dist, torch), own, \
            etas.size

    for s in range(args.warmup):
        step(s, False)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    own = E = 0
    for s in range(args.steps):
        last, own, E = step(args.warmup + s, True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dt, world, dist, torch)
    K = args.steps
    red = acc['reduce_ms'] / K
    flops_red = 4.0 * n ** 3 / 3.0
    total = args.eta_total if args.scaling == 'strong' else world * E
    out = {
        'value': total * K / dt, 'unit': 'evals/s', 'ms_per_step': dt / K * 1e3,
        'eta_per_rank_per_step': E,
        'step': 'band reduction of K (Q^T [X z] applied alongside; repeated on every rank, '
                'the setup does not shard) + %d banded Cholesky evals per rank + host lp + '
                'all-gather' % E,
        'reduce_ms': round(red, 3), 'rhs_ms': round(acc['rhs_ms'] / K, 3),
        'loglik_ms': round(acc['loglik_ms'] / K, 3),
        'marginal_evals_per_s_per_gpu': round(E / (acc['loglik_ms'] / K * 1e-3), 1),
        'reduction_tflops': round(flops_red / (red * 1e-3) / 1e12, 3),
        'reduction_mfma_frac': round(flops_red / (red * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
        'panel': b.stats(),
        'lp_sample': [float(v) for v in last[0].tolist()],
        'curve_sha256': curve_sha(last),
        'lp_all_finite': bool(numpy.all(numpy.isfinite(last[:, 1:]))),
    }
    ld_err, lp_err = golden_errors(lambda e: op.loglik_terms(e, X, z), args.nu, n, m)
    out['logdet_rel_err_vs_reference'] = ld_err
    out['lp_rel_err_vs_reference'] = lp_err
    if ld_ref is not None:
        out['logdet_rel_err_vs_cholesky'] = float(numpy.max(
            numpy.abs(op.loglik_terms(ld_ref[0], X, z)[0] - ld_ref[1]) / numpy.abs(ld_ref[1])))
    if world == 1 and args.scaling == 'strong':
        out['batch_efficiency'] = band_batch_efficiency(op, X, z)
    if not args.no_der:
        out['der1_sweep'] = der1_sweep(op, X, z, E, rank, torch)
    return out, op


def optimizer_timing(D, X, z):
    """The reference's end-to-end task at this N: Likelihood(X, K, method)
    .maximize_log_likelihood(z) (likelihood.py:67-102) for 'direct' (trust-exact
    on lp, jacobian, hessian; _direct_likelihood.py:346-405) and 'profiled'
    (bracket search + Chandrupatla on der1; _profile_likelihood.py:244-415),
    from the resident K: the operator's band reduction and every evaluation
    included (traceinv of exponents 1 and 2 by selected inversion of each
    evaluation's factor, so no eigenvalue chase: band_eigenvalue_calls counts
    them). Wall time and the optimum."""
    import contextlib
    import io
    from gaussian_proc._likelihood import Likelihood
    from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood
    from gaussian_proc import _hip
    out = {}
    for method in ('direct', 'profiled'):
        torch_sync()
        eig0 = _hip.Band.eigenvalue_calls
        t0 = time.perf_counter()
        lik = Likelihood(X, D, method)
        with contextlib.redirect_stdout(io.StringIO()) as buf:
            res = lik.maximize_log_likelihood(z)
        dt = time.perf_counter() - t0
        entry = {'wall_s': round(dt, 3),
                 'result': {k: (float(v) if not isinstance(v, bool) else v)
                            for k, v in res.items()},
                 # traceinv of exponents 1 and 2 by selected inversion: no eigenvalue
                 # chase on either optimizer's path (round 6)
                 'band_eigenvalue_calls': _hip.Band.eigenvalue_calls - eig0}
        if method == 'profiled':
            calls, points, _ = ProfileLikelihood.last_der1_calls
            entry['der1_device_calls'] = calls
            entry['der1_points'] = points
        else:
            txt = buf.getvalue()
            entry['optimizer'] = [l for l in txt.splitlines() if l.startswith('Iter')][-1:]
        lik.K_mixed.band().close()
        out[method] = entry
    return out


def torch_sync():
    import torch
    torch.cuda.synchronize()


def dense_slq_mode(D, etas, ld_exact, nprobe=20, steps=30, tol=1e-3, reps=3):
    """imate 'slq' on the resident dense K (gpmi_sp_create_dense): the logdet
    curve over the same eta grid from ONE device Lanczos of nprobe probes (K X on
    fp64 MFMA, dense_mm_kernel: 8 n^2 bytes of K per product, HBM-bound), with
    imate's ``lanczos_tol`` = tol: the degree doubles from ``steps`` until the
    Gauss / Gauss-Radau gap of the probe-mean logdet quadrature at min(eta) is
    within tol (MixedCorrelation.slq_converge; at N = 16384, nu = 1.5 the smooth
    K needs ~240 steps at eta = 1e-3, where 30 steps left a 22 % bias). Checked
    against the dense Cholesky logdets of the headline line in standard errors of
    the probe mean. ``value``: the curve at the converged degree, degree search
    included (``search_ms``) and alone at that degree (``curve_ms``). A
    logdet-curve leg, not an lp: the likelihood's Gram blocks still take the
    exact solves (_linear_solver.py:71)."""
    from gaussian_proc import _slq
    from gaussian_proc._mixed_correlation import MixedCorrelation
    # full reorthogonalisation: the plain recurrence (imate's default) had not converged
    # at 256 steps at eta = 1e-3 on this smooth K (Gauss / Gauss-Radau gap 1.6e-2,
    # 7.3 standard errors off)
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': nprobe, 'lanczos_degree': steps,
                                         'lanczos_tol': tol, 'orthogonalize': -1})
    n = op.n
    torch_sync()
    t0 = time.perf_counter()
    conv = op.slq_converge(etas)
    per = n * _slq.quadrature(op.slq_nodes(), etas, numpy.log)
    t_search = time.perf_counter() - t0
    deg = conv['degree']
    fixed = MixedCorrelation(D, imate_method='slq',
                             imate_options={'num_samples': nprobe, 'lanczos_degree': deg,
                                            'orthogonalize': -1})
    times = []
    for r in range(reps):
        fixed._lz = None
        t0 = time.perf_counter()
        per_f = n * _slq.quadrature(fixed.slq_nodes(), etas, numpy.log)
        times.append(time.perf_counter() - t0)
    t = float(numpy.median(times))
    est = per.mean(axis=0)
    se = per.std(axis=0, ddof=1) / numpy.sqrt(nprobe)
    mm = {w: op.sop.bench_spmm(w, 10) for w in sorted({16, nprobe, 32})}
    mm_ms = mm[nprobe]
    kbytes = 8.0 * n * n
    out = {'value': round(len(etas) / t_search, 1), 'unit': 'logdet evals/s',
           'value_at_fixed_degree': round(len(etas) / t, 1),
           'search_ms': round(t_search * 1e3, 3), 'curve_ms': round(t * 1e3, 3),
           'etas': len(etas), 'probes': nprobe, 'lanczos_degree_start': steps,
           'lanczos_tol': tol, 'convergence': conv,
           'fixed_degree_curve_equal': bool(numpy.array_equal(per_f, per)),
           'kernel': op.sop.spmm_kernel(nprobe),
           'dense_mm': {'avg_launch_ms': round(mm_ms, 4), 'bytes': kbytes,
                        'gbs': round(kbytes / (mm_ms * 1e-3) / 1e9, 1),
                        'hbm_frac': round(kbytes / (mm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        'ms_by_columns': {str(w): round(v, 4) for w, v in mm.items()}}}
    if ld_exact is not None:
        zs = (est - ld_exact) / se
        pick = [0, int(numpy.argmin(numpy.abs(numpy.log(etas)))), len(etas) - 1]
        out['logdet_check'] = {
            'eta': [float(etas[i]) for i in pick],
            'rel_err': [float(abs(est[i] - ld_exact[i]) / abs(ld_exact[i])) for i in pick],
            'err_in_std_errors': [round(float(zs[i]), 3) for i in pick],
            'max_abs_std_errors_all_eta': round(float(numpy.max(numpy.abs(zs))), 3),
            'etas_within_3_std_errors': int(numpy.sum(numpy.abs(zs) <= 3.0))}
    fixed.sop.close()
    op.sop.close()
    return out


def band_nu25_check(D, points, X, z):
    """BASELINE cfg3 as specified (nu = 2.5, smoother, so more nearly rank-deficient
    panels): one band reduction of that K, its panel statistics (CholeskyQR
    panels that fell back to Householder, reductions redone) and the band logdet /
    lp against the reference's N = 16384 nu = 2.5 values (cfg3_nu25.json). The
    resident K is reassembled at nu = 2.5 (the dense measurements are done)."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    n, m = X.shape
    D.op.assemble_matern(points, numpy.full(2, 0.1), 2.5)
    op = MixedCorrelation(D, imate_method='eigenvalue')
    b = op.band()
    op.refresh_band(X, z)
    red = b.last_timing()['reduce_ms']
    ld_err, lp_err = golden_errors(lambda e: op.loglik_terms(e, X, z), 2.5, n, m)
    out = {'reduce_ms': round(red, 3), 'panel': b.stats(),
           'logdet_rel_err_vs_reference': ld_err, 'lp_rel_err_vs_reference': lp_err}
    b.close()
    return out


def dense_nu25_mode(args, op, X, z, steps=3):
    """BASELINE configs[2] as written: the dense 64-eta curve of the N = 16384
    Matern nu = 2.5 K (the resident K reassembled at nu = 2.5 by the caller), one
    warm-up and `steps` timed steps of the same batched factorization as the
    headline, with the logdet / direct lp errors against the reference's
    N = 16384 nu = 2.5 values (tests/golden/cfg3_nu25.json). The Cholesky's cost
    does not depend on nu; this line shows it."""
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms_batch
    n, m = X.shape
    etas = numpy.logspace(-3, 3, args.eta_total)
    op.loglik_terms(etas, X, z)
    torch_sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ld, G = op.loglik_terms(etas, X, z)
        _lp_from_terms_batch(n, m, 1.0, ld, G)
    torch_sync()
    dt = time.perf_counter() - t0
    ld_err, lp_err = golden_errors(lambda e: op.loglik_terms(e, X, z), 2.5, n, m)
    return {'workload': 'cfg3 as specified: N=%d Matern nu=2.5 rho=0.1, the %d-point eta '
                        'curve logspace(-3,3,%d) per step' % (n, etas.size, etas.size),
            'steps': steps, 'warmup': 1, 'ms_per_step': round(dt / steps * 1e3, 2),
            'value': round(etas.size * steps / dt, 3), 'unit': 'evals/s',
            'logdet_rel_err_vs_reference': ld_err, 'lp_rel_err_vs_reference': lp_err}


def band_batch_efficiency(op, X, z, batches=(8, 16, 32, 64)):
    """The band operator's per-rank eta batches of the strong-scaled curve at
    N = 8 / 4 / 2 / 1: device time of the banded-Cholesky call for that batch
    (one workgroup per eta, so 8 eta leave most CUs idle) and the expected
    time-to-curve with the reduction (repeated on every rank, it does not shard)."""
    b = op.band()
    red = b.last_timing()['reduce_ms']
    grid = numpy.logspace(-3, 3, 64)
    out = {}
    for bsz in batches:
        etas = grid[:bsz]
        op.loglik_terms(etas, X, z)
        times = []
        for _ in range(2):
            op.loglik_terms(etas, X, z)
            times.append(b.last_timing()['loglik_ms'])
        best = min(times)
        out[str(bsz)] = {'loglik_ms': round(best, 3),
                         'evals_per_s_after_reduction': round(bsz / (best * 1e-3), 1),
                         'expected_time_to_64_curve_ms_at_N': {
                             str(64 // bsz): round(red + best, 2)}}
    return out


def der1_sweep(op, X, z, E, rank, torch):
    """ProfileLikelihood.log_likelihood_der1_eta over this rank's E points of the
    grid in one call on the band operator right after its reduction: the Gram
    blocks G1..G3 and trace((K + eta I)^-1) from ONE cyclic-reduction factorization
    per eta, the traces by selected inversion down its tree (no eigenvalues:
    `wall_ms` is the whole cost after the reduction). For comparison the round-4
    path: the one-time eigenvalues of K (timed separately) and the eigenvalue sums,
    and the two der1 curves' agreement."""
    from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood
    log_etas = numpy.linspace(-3, 3, 64)[[(rank * E + j) % 64 for j in range(E)]]
    op._eig = None
    ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, op, log_etas)   # warm (buffers)
    op._der_cache = None   # time the device work, not the operator's last-call cache
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d1 = ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, op, log_etas)
    dt = time.perf_counter() - t0
    out = {'etas': E, 'wall_ms': round(dt * 1e3, 3), 'device_ms': round(op.band().der_ms(), 3),
           'selected_inversion_ms': round(op.band().sinv_ms(), 3),
           'der1_evals_per_s_per_gpu': round(E / dt, 1),
           'traceinv': 'selected inversion of the cyclic-reduction factor (no eigenvalues)',
           'der1_sample': [float(log_etas[0]), float(d1[0])]}
    # the eigenvalue path for comparison
    t0 = time.perf_counter()
    op.eigenvalues()
    eig_ms = (time.perf_counter() - t0) * 1e3
    op._der_cache = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d1e = ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, op, log_etas)
    dte = time.perf_counter() - t0
    out['eigenvalue_path'] = {
        'eigenvalues_ms_once': round(eig_ms, 1), 'sweep_wall_ms': round(dte * 1e3, 3),
        'eigenvalues_chase': {2: 'chase_split_kernel (D and E workgroup per position)',
                              1: 'chase_systolic_kernel (one workgroup per position)',
                              0: 'per-wavefront launches'}[op.band().chase_info()['systolic']],
        'der1_diff_vs_selected_inversion_rel_to_max': float(
            numpy.max(numpy.abs(d1e - d1)) / numpy.max(numpy.abs(d1e)))}
    return out


def batch_efficiency(op, X, z, batches=(8, 16, 32)):
    """Single-GPU evals/s of one device call at smaller eta batches: the
    per-rank batch of the strong-scaled 64-eta curve at N = 8, 4, 2, hence the
    expected time-to-curve there (one warm call, then the best of two)."""
    out = {}
    grid = numpy.logspace(-3, 3, 64)
    for bsz in batches:
        if bsz > op.op.max_batch:
            continue
        etas = grid[:bsz]
        op.loglik_terms(etas, X, z)
        best = min(t for t, _ in _timed(lambda: op.loglik_terms(etas, X, z), 2))
        out[str(bsz)] = {'evals_per_s': round(bsz / best, 2), 'call_ms': round(best * 1e3, 2),
                         'expected_time_to_64_curve_ms_at_N': {
                             str(64 // bsz): round(best * 1e3, 2)}}
    return out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv=None):
    """``--gpus N`` (N > 1) started as a plain ``python bench.py --gpus N``: run
    the N ranks, one process per GPU, under ``torch.distributed.run`` as a CHILD
    process (rendezvous on 127.0.0.1), forward its output and return its exit
    code. This process never touches a device (no HIP call before the ranks
    exist, none after), so the launch is the same one the driver makes itself."""
    import subprocess
    argv = sys.argv[1:] if argv is None else list(argv)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.abspath(__file__)] + argv
    log('launching %d ranks: %s' % (args.gpus, ' '.join(cmd[1:])))
    return subprocess.call(cmd)


def rank_devices(args, world, rank, local, dist, torch):
    """Check the launch against ``--gpus`` and name the device every rank uses.
    Fails loudly (SystemExit) when the job's world size is not ``--gpus`` or
    fewer devices are visible than ranks need. Returns the per-rank list
    (gathered at N > 1) for the line's ``devices``."""
    share = os.environ.get('GPMI_BENCH_SHARE_DEVICE') == '1'
    if world != args.gpus:
        raise SystemExit('bench: --gpus %d but the job has %d ranks (WORLD_SIZE)'
                         % (args.gpus, world))
    visible = torch.cuda.device_count()
    need = 1 if share else max(world, local + 1)
    if visible < need:
        raise SystemExit('bench: %d ranks need %d visible devices, %d visible'
                         % (world, need, visible))
    props = torch.cuda.get_device_properties(local)
    me = {'rank': rank, 'local_rank': int(os.environ.get('LOCAL_RANK', '0')), 'device': local,
          'name': props.name, 'pci_bus_id': getattr(props, 'pci_bus_id', None),
          'uuid': str(getattr(props, 'uuid', '')), 'host': platform.node(),
          'shared_device': share}
    if dist is None:
        return [me]
    out = [None] * world
    dist.all_gather_object(out, me)
    if not share and world > 1:
        ids = {(d['host'], d['uuid'] or d['device']) for d in out}
        if len(ids) != world:
            raise SystemExit('bench: ranks share a device: %s' % out)
    return out


def launch_check(args, world, rank, torch):
    """``--launch-check``: the multi-rank plumbing of the line without a device
    (CPU box, gloo): the world size against --gpus, each rank's eta block of the
    strong-scaled curve, the ONE all-gather of the rows and the max-over-ranks
    time. Rank 0 prints {n_gpus, ranks, curve_etas, ...}."""
    dist = None
    if world > 1:
        dist = torch.distributed
        dist.init_process_group('gloo')
    if world != args.gpus or (dist is not None and dist.get_world_size() != args.gpus):
        raise SystemExit('bench: --gpus %d but the job has %d ranks' % (args.gpus, world))
    from gaussian_proc.sweep import shard
    t0 = time.perf_counter()
    etas, own, per, gsize = eta_block(args, world, rank)
    rows = numpy.stack([etas, numpy.full(per, float(rank)), numpy.arange(per, dtype=float)],
                       axis=1)
    if dist is None:
        allrows = rows
    else:
        from gaussian_proc.sweep import _all_gather_rows
        allrows = _all_gather_rows(dist, None, rows, world)
    dt = max_over_ranks(time.perf_counter() - t0, world, dist, torch)
    owns = [shard(gsize, world, r)[1] - shard(gsize, world, r)[0] for r in range(world)] \
        if args.scaling == 'strong' else [per] * world
    curve = numpy.concatenate([allrows[r * per:r * per + owns[r], 0] for r in range(world)])
    if rank == 0:
        print(json.dumps({'launch_check': True, 'n_gpus': world, 'gpus_arg': args.gpus,
                          'ranks': sorted({int(v) for v in allrows[:, 1]}),
                          'eta_per_rank': per, 'curve_etas': curve.tolist(),
                          'max_rank_s': dt}), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit('bench: --gpus must be >= 1')
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # plain `python bench.py --gpus N`: start the N ranks (child process)
        sys.exit(launch_ranks(args))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch
    import torch.distributed
    if args.launch_check:
        return launch_check(args, world, rank, torch)
    # one process per GPU over RCCL; GPMI_BENCH_BACKEND=gloo with
    # GPMI_BENCH_SHARE_DEVICE=1 rehearses the N>1 flow with every rank on
    # device 0 (the one-GPU box), host-side collectives. GPMI_BENCH_PG=1 creates
    # the process group (and its collectives) at N = 1 too: the RCCL
    # communicator's streams beside the measured kernels, on one GPU
    backend = os.environ.get('GPMI_BENCH_BACKEND', 'nccl')
    if os.environ.get('GPMI_BENCH_SHARE_DEVICE') == '1':
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1 or os.environ.get('GPMI_BENCH_PG') == '1':
        dist = torch.distributed
        if world == 1:
            # a one-rank group of a plain `python bench.py` (env:// rendezvous)
            for k, v in (('RANK', '0'), ('WORLD_SIZE', '1'), ('MASTER_ADDR', '127.0.0.1'),
                         ('MASTER_PORT', str(_free_port()))):
                os.environ.setdefault(k, v)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise SystemExit('bench: process group has %d ranks, WORLD_SIZE %d'
                             % (dist.get_world_size(), world))
    devices = rank_devices(args, world, rank, local, dist, torch)

    if args.config != 'dense':
        return run_sparse(args, world, rank, local, dist, torch, devices)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    from gaussian_proc import generate_correlation, _data
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms, _lp_from_terms_batch

    points = _data.generate_points(args.grid, 2, True)
    z = _data.generate_data(points, 0.2)
    X = _data.generate_basis_functions(points, 2)
    n, m = X.shape
    _, own, B, gsize = eta_block(args, world, rank)
    max_batch = max(B, 64 if world == 1 else B)
    D = generate_correlation(points, 0.1, args.nu, device_resident=True, device=local,
                             max_batch=max_batch)
    from gaussian_proc import _hip
    asm_cold_ms = _hip.last_assembly_ms()     # first launch (code load, first touch)
    D.op.assemble_matern(points, numpy.full(2, 0.1), args.nu)   # same K again, warm
    asm_ms = _hip.last_assembly_ms()
    asm_bytes = 8.0 * D.op.n_pad ** 2
    op = MixedCorrelation(D)
    op.op.set_outer(args.outer)
    op.set_rhs(X, z)

    def step(s, timing_acc=None):
        etas = eta_block(args, world, rank, s)[0]
        ld, G = op.loglik_terms(etas, X, z)
        if timing_acc is not None:
            t = op.op.last_timing()
            for k in ('syrk_ms', 'syrk_busy_ms', 'syrk_flops', 'syrk_launches', 'total_ms'):
                timing_acc[k] += t[k]
        lp = _lp_from_terms_batch(n, m, 1.0, ld, G)
        return gather_rows(numpy.stack([etas, ld, lp], axis=1), world, dist, torch)

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
    dt = max_over_ranks(dt, world, dist, torch)
    log('dense: %d steps in %.2f s' % (args.steps, dt))
    # evaluations the job completed: the whole curve per step (strong), or every
    # rank's block (weak)
    evals = (gsize if args.scaling == 'strong' else world * B) * args.steps
    flops_eval = n ** 3 / 3.0 + 2.0 * n ** 2 * (m + 1) + n ** 2
    result = None
    if rank == 0:
        roof = None
        if not args.no_timing and timing['syrk_ms'] > 0:
            # algorithmic flops per launch / average launch duration (HIP events on
            # the launching stream) = total flops / summed launch time. A batch of
            # <= 32 (N >= 2 ranks) runs as two halves on two streams whose SYRK
            # launches overlap: there the summed durations overcount the time and
            # the union of the launch intervals (busy_ms) is the divisor
            overlapped = B <= 32 and os.environ.get('GPMI_GROUPS', '0') in ('0', '2')
            div_ms = timing['syrk_busy_ms'] if overlapped else timing['syrk_ms']
            achieved = timing['syrk_flops'] / (div_ms * 1e-3) / 1e12
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
                    'batch_streams': 2 if overlapped else 1,
                    'per_launch_tflops': round(timing['syrk_flops'] / (timing['syrk_ms'] * 1e-3)
                                               / 1e12, 3)}
        whole = flops_eval * evals / world / dt / 1e12
        if args.scaling == 'strong':
            workload = ('cfg3: N=%d 2D grid Matern nu=%g rho=0.1, the %d-point eta curve '
                        'logspace(-3,3,%d) per step, %d eta per rank' % (n, args.nu, gsize, gsize, B))
        else:
            workload = ('cfg3 grid, weak: N=%d 2D grid Matern nu=%g rho=0.1, %d eta per rank of '
                        'logspace(-3,3,%d)' % (n, args.nu, B, gsize))
        result = {
            'metric': 'log-likelihood evals/sec (N=16384 dense Matern-3/2)',
            'value': evals / dt,
            'unit': 'evals/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': dt / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': args.scaling,
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic (reference data_utilities: 2D grid, sin + 0.2 noise seed 31, '
                    'deg-2 basis)',
            'config': {'workload': workload, 'n': n, 'm': m, 'eta_per_rank_per_step': B,
                       'operator': "imate_method='cholesky' (one dense fp64 MFMA Cholesky per "
                                   "eta); band_mode below is the 'eigenvalue' operator "
                                   "Likelihood uses",
                       'outer_panel': 128 * args.outer,
                       'parallelism': 'eta-shard x%d + all-gather' % world},
            'roofline': roof,
            'whole_eval_tflops_per_gpu': round(whole, 3),
            'whole_eval_mfma_frac': round(whole / FP64_MFMA_PEAK_TFLOPS, 4),
            'flops_per_eval': flops_eval,
            'lp_sample': [float(v) for v in last[0].tolist()] if last is not None else None,
            'curve_sha256': curve_sha(last) if last is not None else None,
            'lp_all_finite': (bool(numpy.all(numpy.isfinite(last[:, 1:])))
                              if last is not None else None),
            'cpu_baseline': None,
            'devices': devices,
        }
        if args.scaling == 'strong':
            result['time_to_curve_ms'] = dt / args.steps * 1e3
        # one-time dense assembly (HBM-write-bound, 8 n^2 bytes)
        result['assembly'] = {'kernel': 'matern_dense_kernel (64x64 lower tiles, mirrored)',
                              'ms': round(asm_ms, 4), 'first_call_ms': round(asm_cold_ms, 4),
                              'bytes_written': asm_bytes,
                              'gbs': round(asm_bytes / (asm_ms * 1e-3) / 1e9, 1),
                              'hbm_frac': round(asm_bytes / (asm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                                4)}
    ld_err, lp_err = golden_errors(lambda e: op.loglik_terms(e, X, z), args.nu, n, m)
    if rank == 0:
        result['logdet_rel_err_vs_reference'] = ld_err
        result['lp_rel_err_vs_reference'] = lp_err
        if world == 1 and args.scaling == 'strong' and not args.no_extras:
            result['batch_efficiency'] = batch_efficiency(op, X, z)
            # (before band_nu25_check reassembles the resident K at nu = 2.5)
            if last is not None:
                result['dense_slq_mode'] = dense_slq_mode(D, last[:, 0], last[:, 1])
                log('dense slq: %s' % result['dense_slq_mode'])
    lam = None
    if not args.no_band:
        ld_ref = (last[:own, 0], last[:own, 1])
        bm, bop = band_mode(args, D, X, z, world, rank, dist, torch, ld_ref)
        log('band mode: %.1f evals/s' % bm['value'])
        if rank == 0:
            result['band_mode'] = bm
        if bop._eig is not None:
            lam = bop._eig
    lp_dev = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the evaluation the CPU baseline repeats, on the device (eta = 1)
        ld1, G1 = op.loglik_terms([1.0], X, z)
        lp_dev = _lp_from_terms(n, m, 1.0, ld1[0], G1[0])
    if rank == 0 and world == 1 and not args.no_band:
        result['band_mode']['optimizer'] = optimizer_timing(D, X, z)
    if rank == 0 and world == 1 and args.nu == 1.5 and not args.no_extras:
        # BASELINE cfg3 as written (nu = 2.5): the band reduction's check reassembles
        # the resident K at nu = 2.5, then the dense 64-eta curve is timed on it
        if not args.no_band:
            result['band_mode']['nu25_check'] = band_nu25_check(D, points, X, z)
        else:
            D.op.assemble_matern(points, numpy.full(2, 0.1), 2.5)
        result['dense_nu25'] = dense_nu25_mode(args, op, X, z)
        log('dense nu=2.5: %s' % result['dense_nu25'])
    if not args.no_sparse:
        # release the dense and band operators (their streams count against the
        # process's hardware queues) before the sparse configs run
        if not args.no_band:
            bop.band().close()
        op.op.close()
        sm = sparse_modes(args, world, rank, local, dist, torch)
        if rank == 0:
            result['sparse_modes'] = sm
    if lp_dev is not None:
        # after every device measurement (its thread pool's leftovers slow the launch-bound
        # sparse steps); CPU and GPU agree on the same evaluation
        cb = cpu_baseline(points, z, X, args.nu, 1.0, lam, args.cpu_samples)
        cb['lp_rel_diff_vs_device'] = abs(cb['lp_cholesky'] - lp_dev) / abs(lp_dev)
        result['cpu_baseline'] = cb
        result['speedup_vs_cpu'] = round(result['value'] / cb['value'], 1)
    if rank == 0:
        emit(args, result)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
