"""eta-grid sweep of the log-likelihood, sharded over GPUs.

The reference evaluates its likelihood curves point by point on one CPU
(_profile_likelihood.py:567-596 over 100-170 eta values;
_direct_likelihood.py:420-426 over a 20 x 20 grid). Every point is independent
and uses the same K, so the grid is partitioned: rank r of a
``torch.distributed`` group (one process per GPU, backend "nccl" = RCCL over
xGMI) evaluates a contiguous block of eta values with its own device-resident
K (assembled locally from the points: no K broadcast), batched
``max_batch`` per device call; ONE all-gather collects the
[logdet, lp] rows of every rank. Without a process group the whole grid runs
on the local device.
"""

import math

import numpy

from ._likelihood._direct_likelihood import _lp_from_terms

__all__ = ['shard', 'eta_sweep', 'slq_sweep', 'der1_sweep', 'slq_gram_sweep']


def shard(num, world, rank):
    """Contiguous block [lo, hi) of ``num`` items owned by ``rank`` (padded blocks)."""
    per = int(math.ceil(num / float(world)))
    lo = min(num, rank * per)
    hi = min(num, lo + per)
    return lo, hi, per


def _group(group):
    """(dist module or None, world, rank) of an initialised process group."""
    if group is False:
        return None, 1, 0
    try:
        import torch.distributed as dist_mod
        if dist_mod.is_available() and dist_mod.is_initialized():
            return dist_mod, dist_mod.get_world_size(group), dist_mod.get_rank(group)
    except ImportError:
        pass
    return None, 1, 0


def _all_gather_rows(dist, group, local, world):
    """ONE all-gather of equally shaped float64 row blocks -> [world * rows, ...]."""
    import torch
    backend = dist.get_backend(group)
    dev = torch.device('cuda', torch.cuda.current_device()) if backend == 'nccl' \
        else torch.device('cpu')
    t_local = torch.from_numpy(numpy.ascontiguousarray(local)).to(dev)
    if backend == 'nccl':
        t_all = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]),
                            dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(t_all, t_local, group=group)
    else:
        parts = [torch.empty_like(t_local) for _ in range(world)]
        dist.all_gather(parts, t_local, group=group)
        t_all = torch.cat(parts)
    return t_all.cpu().numpy()


def der1_sweep(K_mixed, X, z, log_etas, group=False):
    """ProfileLikelihood.log_likelihood_der1_eta (_profile_likelihood.py:91-132)
    at many log10(eta): each rank evaluates its contiguous block in one batched
    call (band Gram blocks on the eigenvalue operator), ONE all-gather collects
    them. Returns der1[len(log_etas)] on every rank.

    Sharding is opt-in (``group`` None = the default process group, or a
    group): every rank of it must hold the same K, X, z and call this with the
    same log_etas. A rank whose block raises ``LinAlgError`` (K + eta I not
    positive definite there) still joins the all-gather with an error flag in
    its rows, and then every rank raises together."""
    from ._likelihood._profile_likelihood import ProfileLikelihood
    log_etas = numpy.atleast_1d(numpy.asarray(log_etas, dtype=float))
    dist, world, rank = _group(group)
    lo, hi, per = shard(log_etas.size, world, rank)
    local = numpy.zeros((per, 2))
    err = None
    if hi > lo:
        try:
            local[:hi - lo, 0] = ProfileLikelihood.log_likelihood_der1_eta_batch(
                z, X, K_mixed, log_etas[lo:hi])
        except numpy.linalg.LinAlgError as e:
            if dist is None or world == 1:
                raise
            err = e
            local[:, 1] = 1.0
    if dist is None or world == 1:
        return local[:log_etas.size, 0].copy()
    allv = _all_gather_rows(dist, group, local, world)
    if err is not None:
        raise err
    if allv[:, 1].any():
        raise numpy.linalg.LinAlgError(
            'K + eta I is not positive definite at an eta of another rank\'s block')
    return allv[:log_etas.size, 0].copy()


def eta_sweep(K_mixed, X, z, etas, sigma=1.0, group=None):
    """Direct log-likelihood along the eta grid at fixed sigma (sigma0 = sqrt(eta) sigma).

    Returns (logdet[neta], lp[neta]) on every rank."""
    etas = numpy.asarray(etas, dtype=float)
    n, m = X.shape
    dist, world, rank = _group(group)
    lo, hi, per = shard(etas.size, world, rank)
    local = numpy.zeros((per, 2))
    if hi > lo:
        ld, G = K_mixed.loglik_terms(etas[lo:hi], X, z)
        local[:hi - lo, 0] = ld
        local[:hi - lo, 1] = [_lp_from_terms(n, m, sigma, l, g) for l, g in zip(ld, G)]
    if dist is None or world == 1:
        return local[:etas.size, 0].copy(), local[:etas.size, 1].copy()
    allv = _all_gather_rows(dist, group, local, world)[:etas.size]
    return allv[:, 0].copy(), allv[:, 1].copy()


def slq_sweep(K_mixed, etas, group=None, converge=('logdet',)):
    """Stochastic-Lanczos-quadrature curves over an eta grid for a sparse
    ``MixedCorrelation`` (imate_method 'slq'), probes sharded over the ranks.

    Rank r runs the device Lanczos for the probe block [lo, hi) of the global
    probe set (counter-based probes: the union over ranks is exactly the
    single-GPU probe set), evaluates its per-probe quadrature for every eta, and
    ONE all-gather collects the [probe, eta] blocks. Returns
    dict(logdet, traceinv, traceinv2), each [neta], identical on every rank.

    With the operator's ``lanczos_tol`` set, each probe row also carries its Gauss
    and Gauss-Radau quadratures of ``converge`` at min(etas); while their
    probe-mean gap (_slq.bracket) exceeds lanczos_tol, every rank redoes its
    shard at a higher degree (_next_degree, up to max_lanczos_degree) and gathers
    again. The
    decision is taken from the gathered rows, so all ranks agree."""
    from . import _slq
    from ._mixed_correlation.mixed_correlation import _next_degree
    etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
    s = K_mixed.num_samples
    dist, world, rank = _group(group)
    lo, hi, per = shard(s, world, rank)
    names = ('logdet', 'traceinv', 'traceinv2')
    tol = getattr(K_mixed, 'lanczos_tol', None)
    conv = [_slq.FUNCS[f] if isinstance(f, str) else f for f in converge] if tol else []
    lower = K_mixed._lower_bound() if tol else None
    deg = getattr(K_mixed, 'lanczos_degree_used', K_mixed.lanczos_degree)
    # per probe row: the quadratures, the smallest Ritz value (the SPD check runs
    # after the all-gather, on every rank alike: no rank raises alone), the
    # Gauss / Gauss-Radau pair of each converge function at min(etas), and an
    # error flag (a host-side failure of this rank's rows is raised on every rank
    # after the all-gather, not by this rank alone inside the collectives)
    nq = len(names) * etas.size
    ncol = nq + 1 + 2 * len(conv) + 1
    seen = []
    while True:
        local = numpy.zeros((per, ncol))
        local[:, nq] = numpy.inf
        err = None
        if hi > lo:
            a, b = K_mixed.sop.lanczos(hi - lo, deg, K_mixed.seed, probe_offset=lo,
                                       orthogonalize=getattr(K_mixed, 'orthogonalize', 0))
            try:
                nodes = _slq.nodes(a, b)
                q = numpy.empty((hi - lo, len(names), etas.size))
                for f, name in enumerate(names):
                    with numpy.errstate(invalid='ignore', divide='ignore'):
                        q[:, f] = _slq.quadrature(nodes, etas, _slq.FUNCS[name], check=False)
                local[:hi - lo, :nq] = q.reshape(hi - lo, nq)
                local[:hi - lo, nq] = [float(t.min()) for t, _ in nodes]
                if conv:
                    # the node from this rank's Ritz values; radau_nodes never raises
                    node, _ = _slq.radau_node(lower, nodes, etas)
                    radau = _slq.radau_nodes(a, b, node)
                    e = [float(etas.min())]
                    for i, fn in enumerate(conv):
                        with numpy.errstate(invalid='ignore', divide='ignore'):
                            local[:hi - lo, nq + 1 + 2 * i] = _slq.quadrature(
                                nodes, e, fn, check=False)[:, 0]
                            local[:hi - lo, nq + 2 + 2 * i] = _slq.quadrature(
                                radau, e, fn, check=False)[:, 0]
            except (ValueError, numpy.linalg.LinAlgError) as exc:
                if dist is None or world == 1:
                    raise
                err = exc
                local[:, -1] = 1.0
        if dist is not None and world > 1:
            allv = _all_gather_rows(dist, group, local, world)[:s]
            if err is not None:
                raise err
            if allv[:, -1].any():
                raise numpy.linalg.LinAlgError(
                    'slq_sweep: another rank\'s probe shard failed on the host')
        else:
            allv = local[:s]
        _slq.check_shifts(float(allv[:, nq].min()), etas)
        if not conv:
            break
        gap = 0.0
        for i in range(len(conv)):
            g = allv[:, nq + 1 + 2 * i].mean()
            r = allv[:, nq + 2 + 2 * i].mean()
            gap = max(gap, float(_slq.gap(g, r)))   # inf for a NaN rule: not converged
        if gap <= tol or deg >= K_mixed.max_lanczos_degree:
            break
        seen.append((deg, gap))
        deg = min(K_mixed.max_lanczos_degree, _next_degree(seen, tol))
    if conv:
        K_mixed.lanczos_degree_used = deg
        # rigorous: the Radau node is the proven lower bound (_slq.radau_node's flag:
        # lower + min(etas) > 0, the same on every rank), not a Ritz-value heuristic
        rigorous = bool(lower + float(etas.min()) > 0.0)
        K_mixed.last_slq_convergence = {'degree': deg, 'bracket': gap, 'converged': gap <= tol,
                                        'eta': float(etas.min()), 'rigorous_bound': rigorous}
    allq = allv[:, :nq].reshape(s, len(names), etas.size)
    n = K_mixed.n
    return {name: n * allq[:, f].mean(axis=0) for f, name in enumerate(names)}


_CG_POOL = None


def _cg_worker():
    """The one host thread that runs the multi-shift CG beside the Lanczos
    (slq_gram_sweep), created once per process: a thread pool made per sweep cost a
    thread start and join in every likelihood step."""
    global _CG_POOL
    if _CG_POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _CG_POOL = ThreadPoolExecutor(1, thread_name_prefix='gpmi-msgram')
    return _CG_POOL


def slq_gram_sweep(K_mixed, etas, R, rtol=1e-6, group=None, split='columns'):
    """One sparse likelihood sweep: slq_sweep (the Lanczos of this rank's probe
    shard, all-gathered quadratures) and the multi-shift CG Gram blocks
    R^T (K + eta I)^-1 R (_linear_solver.py:57-68 at ``rtol``), run TOGETHER: the
    Gram on a second host thread, whose device calls go to the multi-shift CG's own
    stream (gpmi_sp_msgram), beside the Lanczos on the operator's stream. The two
    are independent (the same K, different vectors), and each alone leaves the
    device partly idle (latency-bound scalar and reduction launches).

    On several ranks the Gram is split by right-hand-side columns (``split=
    'columns'``, default): rank r solves its column shard of R for EVERY eta
    (gpmi_sp_msgram_cols, dotted with all of R) and one all-gather after the
    Lanczos's collects the columns, so each rank runs a fraction of the CG's SpMMs.
    ``split='eta'`` gives each rank the full CG for its eta block (the per-shift
    scalars only divide).

    ``R = None``: the right-hand sides K_mixed.sop.set_rhs made resident in HBM.

    Returns (curves, (lo, hi), G[hi - lo, s, s]): slq_sweep's curves on every
    rank, and this rank's contiguous eta block with its Gram blocks.

    The multi-shift CG's negative-curvature check (``LinAlgError``) depends on
    the right-hand sides, so on several ranks it can fire on one rank only: that
    rank still joins the collectives with an error flag, and every rank raises
    after them (as der1_sweep)."""
    etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
    if R is None:
        # the block K_mixed.sop.set_rhs made resident in HBM (no upload per sweep)
        R2, s = None, K_mixed.sop.rhs_cols
        if not s:
            raise ValueError('slq_gram_sweep: R is None but no resident block (sop.set_rhs)')
    else:
        R = numpy.asarray(R, dtype=float)
        R2 = R[:, None] if R.ndim == 1 else R
        s = R2.shape[1]
    dist, world, rank = _group(group)
    multi = dist is not None and world > 1
    lo, hi, _ = shard(etas.size, world, rank)
    by_cols = multi and split == 'columns'
    clo, chi, cper = shard(s, world, rank)
    err = None
    ex = _cg_worker()
    if by_cols:
        fut = (ex.submit(K_mixed.sop.msgram, etas, R2, rtol, None, (clo, chi))
               if chi > clo else None)
    else:
        fut = ex.submit(K_mixed.sop.msgram, etas[lo:hi], R2, rtol) if hi > lo else None
    try:
        curves = slq_sweep(K_mixed, etas, group=group)
    finally:
        try:
            G = fut.result() if fut is not None else None
        except numpy.linalg.LinAlgError as e:
            if not multi:
                raise
            err, G = e, None
    if by_cols:
        # one row per column c (its G[:, :, c] flattened) plus an error flag, cper
        # rows per rank; the all-gather runs after the Lanczos's (collectives in the
        # same order on every rank, from the main thread)
        local = numpy.zeros((cper, etas.size * s + 1))
        if G is not None:
            local[:chi - clo, :-1] = G.transpose(2, 0, 1).reshape(chi - clo, -1)
        if err is not None:
            local[:, -1] = 1.0
        allv = _all_gather_rows(dist, group, local, world)
        flags = allv[:, -1]
        allv = allv[:, :-1]
    elif multi:
        # the eta split has no collective of its own: one flag per rank
        flags = _all_gather_rows(dist, group, numpy.array([[1.0 if err else 0.0]]), world)
    if multi:
        if err is not None:
            raise err
        if flags.any():
            raise numpy.linalg.LinAlgError(
                'K + eta I is not positive definite: negative curvature in another '
                'rank\'s multi-shift CG')
    if by_cols:
        Gf = numpy.empty((etas.size, s, s))
        for r in range(world):
            a, b, _ = shard(s, world, r)
            if b > a:
                blk = allv[r * cper:r * cper + (b - a)].reshape(b - a, etas.size, s)
                Gf[:, :, a:b] = blk.transpose(1, 2, 0)
        G = Gf[lo:hi] if hi > lo else None
    return curves, (lo, hi), G
