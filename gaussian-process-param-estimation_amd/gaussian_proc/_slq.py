"""Stochastic Lanczos quadrature on top of the device Lanczos (gpmi_sp_lanczos).

The published SLQ estimator that imate's 'slq' method implements
(mixed_correlation.py:138-143,204-209,263-268 call it through
``imate.AffineMatrixFunction``): with Rademacher probes v_1..v_s and the
Lanczos tridiagonal T_k of K started at v_p / |v_p| with Ritz pairs
(theta_i, e_1-components tau_i),

    tr f(K + eta I) ~= n / s * sum_p sum_i tau_pi^2 f(theta_pi + eta).

The Krylov space of K + eta I does not depend on eta, so one Lanczos run per
probe serves every eta (the AffineMatrixFunction property). Probes are
counter-based (seed, global probe index), so a probe set split over GPUs is
identical to the single-GPU one.
"""

import numpy
import scipy.linalg


def _length(b):
    """Order of a probe's tridiagonal: up to its first zero beta (breakdown:
    the Krylov space is invariant and the Gauss rule exact) or all steps."""
    z = numpy.flatnonzero(b == 0.0)
    return int(z[0]) + 1 if z.size else len(b)


def _rule(d, e):
    """Nodes and squared first eigenvector components of the symmetric
    tridiagonal (diagonal d, off-diagonal e): LAPACK stemr through scipy; the
    dense symmetric solver where stemr does not converge (tight clusters: the
    duplicated Ritz values of a recurrence without reorthogonalisation)."""
    if d.size == 1:
        return d.copy(), numpy.ones(1)
    try:
        theta, U = scipy.linalg.eigh_tridiagonal(d, e)
    except numpy.linalg.LinAlgError:
        theta, U = numpy.linalg.eigh(numpy.diag(d) + numpy.diag(e, 1) + numpy.diag(e, -1))
    return theta, U[0] ** 2


def nodes(alpha, beta):
    """Ritz values and squared first components for each probe (the Gauss
    quadrature rule of the probe's spectral measure).
    alpha, beta: [nprobe, steps]; beta[p, k] = 0 ends probe p's tridiagonal
    after step k; beta[p, steps - 1] is the coupling beta_m of the last Lanczos
    vector to the next one (used by radau_nodes only).
    The probes whose tridiagonal runs the full length (no breakdown: every probe of
    a sweep, as a rule) are solved together by one batched dense symmetric
    eigensolver call (numpy.linalg.eigh on the [nprobe, k, k] stack: one call
    instead of one scipy call per probe, half the host time of a cfg 4 / cfg 5 step's
    20 probes); the others one by one (_rule). The solver of a probe depends only
    on its own tridiagonal, never on how many probes share the call (a rank's
    shard of one probe, or the adaptive extra batches, get the nodes the whole set
    gives it at N = 1)."""
    alpha = numpy.asarray(alpha, dtype=float)
    beta = numpy.asarray(beta, dtype=float)
    lens = [_length(b) for b in beta]
    out = [None] * len(lens)
    full = [p for p, k in enumerate(lens) if k == alpha.shape[1] and k > 1]
    if full:
        k = alpha.shape[1]
        T = numpy.zeros((len(full), k, k))
        i = numpy.arange(k)
        T[:, i, i] = alpha[full]
        T[:, i[:-1], i[1:]] = beta[full, :k - 1]
        T[:, i[1:], i[:-1]] = beta[full, :k - 1]
        theta, U = numpy.linalg.eigh(T)
        for q, p in enumerate(full):
            out[p] = (theta[q], U[q, 0] ** 2)
    for p, k in enumerate(lens):
        if out[p] is None:
            out[p] = _rule(alpha[p, :k], beta[p, :k - 1])
    return out


def _last_pivot(a, b, lower):
    """Last pivot d_m of (T_m - lower I) = L D L^T (T_m: diagonal a, off-diagonal b)."""
    d = a[0] - lower
    for i in range(1, a.size):
        d = (a[i] - lower) - b[i - 1] ** 2 / d
    return d


def radau_nodes(alpha, beta, lower):
    """Gauss-Radau rules with one node fixed at ``lower`` <= lambda_min(K)
    (Golub and Meurant, "Matrices, Moments and Quadrature with Applications",
    2010, ch. 6): the tridiagonal T_m extended by beta_m and the diagonal entry
    a~ = lower + beta_m^2 / d_m, d_m the last pivot of (T_m - lower I) = L D L^T.
    For f with f^(2m) of constant sign on the spectrum (log(x + eta),
    (x + eta)^-p) the Gauss and Gauss-Radau values bracket the exact quadratic
    form, so their gap bounds the Lanczos quadrature error of each probe. A
    probe whose tridiagonal broke down (exact rule) gets its Gauss rule.

    ``lower`` only a hair below a probe's smallest Ritz value can leave the
    pivot d_m <= 0 from rounding alone (T_m - lower I is then numerically
    singular): that probe's node moves down to its own smallest Ritz value minus
    1e-8 max|T_m| (and 1e-6 max|T_m| if that still fails), a node still below its
    rule's nodes. If no node works the probe gets a NaN rule (one node, NaN): its
    Radau quadrature, the probe mean and the bracket are then NaN, which the
    degree searches read as "not converged" (a Gauss rule in its place would give
    the probe a zero gap and could close the bracket falsely). Nothing here
    raises, so a rank of a sharded sweep never leaves the collectives alone
    (sweep.slq_sweep)."""
    out = []
    for a, b in zip(alpha, beta):
        a = numpy.asarray(a, dtype=float)
        b = numpy.asarray(b, dtype=float)
        k = _length(b)
        if k < len(b) or b[k - 1] == 0.0:
            out.append(_rule(a[:k], b[:k - 1]))
            continue
        node = float(lower)
        d = _last_pivot(a[:k], b[:k - 1], node)
        if not d > 0.0:
            theta = _rule(a[:k], b[:k - 1])[0]
            scale = max(float(numpy.max(numpy.abs(a[:k]))),
                        float(numpy.max(numpy.abs(b[:k]))), 1e-300)
            for rel in (1e-8, 1e-6):
                node = min(float(lower), float(theta.min()) - rel * scale)
                d = _last_pivot(a[:k], b[:k - 1], node)
                if d > 0.0:
                    break
        if not d > 0.0:
            out.append((numpy.array([numpy.nan]), numpy.ones(1)))
            continue
        dd = numpy.append(a[:k], node + b[k - 1] ** 2 / d)
        out.append(_rule(dd, b[:k]))
    return out


def radau_node(lower, node_list, etas):
    """The fixed Gauss-Radau node for the quadratures of f(x + eta), eta >= min(etas).

    ``lower`` (a proven lower bound of lambda_min(K): the user's
    spectrum_lower_bound, 0 for a dense correlation matrix, a sparse K's Gershgorin
    bound) is used while f stays finite there, i.e. lower + min(etas) > 0. A sparse
    tapered K's Gershgorin bound is usually far below -min(eta) (log and the
    inverse powers are NaN / infinite at such a node, so the bracket could never
    close): the node is then the smallest Ritz value minus a margin (1e-8 of the
    largest |Ritz value|), or half-way between -min(etas) and that Ritz value if
    the margin would cross -min(etas). That node is a heuristic, not a proven
    bound (lambda_min may lie below the smallest Ritz value); pass
    ``spectrum_lower_bound`` for a rigorous bracket. Returns (node, rigorous)."""
    e0 = float(numpy.min(etas))
    tmin = min_ritz(node_list)
    scale = max((float(numpy.max(numpy.abs(t))) for t, _ in node_list), default=1.0)
    margin = 1e-8 * max(scale, 1e-300)
    if lower + e0 > 0.0:
        return min(float(lower), tmin - margin), True
    node = tmin - margin
    if not node + e0 > 0.0:
        node = 0.5 * (tmin - e0)
    return node, False


def gap(g, r):
    """Relative gap |g - r| / |g| of a Gauss / Gauss-Radau pair (|g - r| for g = 0);
    inf when either is not finite (a probe without a valid Radau node, or f
    undefined at a node): never read as converged."""
    g = numpy.asarray(g, dtype=float)
    r = numpy.asarray(r, dtype=float)
    with numpy.errstate(divide='ignore', invalid='ignore'):
        out = numpy.where(g != 0.0, numpy.abs(g - r) / numpy.abs(g), numpy.abs(g - r))
    return numpy.where(numpy.isfinite(g) & numpy.isfinite(r), out, numpy.inf)


def bracket(gauss, radau, etas, fn):
    """Relative gap |mean_p G_p - mean_p R_p| / |mean_p G_p| of the probe-mean
    Gauss and Gauss-Radau quadratures at each eta: a bound on the Lanczos
    (quadrature) part of the SLQ error, as opposed to its Monte-Carlo part (inf
    when a probe has no valid Radau rule, see radau_nodes)."""
    with numpy.errstate(divide='ignore', invalid='ignore'):
        g = quadrature(gauss, etas, fn, check=False).mean(axis=0)
        r = quadrature(radau, etas, fn, check=False).mean(axis=0)
    return gap(g, r)


def min_ritz(node_list):
    """Smallest Ritz value over the probes (inf for none)."""
    return min((float(t.min()) for t, _ in node_list), default=numpy.inf)


def check_shifts(theta_min, etas):
    """Every K + eta I must be positive definite. Ritz values lie inside
    [lambda_min, lambda_max] of K, so theta_min + eta <= 0 proves that
    K + eta I is not (the tapered Matern is indefinite): raise
    numpy.linalg.LinAlgError, as scipy's posv does on a dense non-SPD matrix."""
    etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
    if etas.size and not theta_min + etas.min() > 0.0:
        raise numpy.linalg.LinAlgError(
            'K + eta I is not positive definite for eta = %r: a Lanczos Ritz value of K '
            'is %r (choose eta > |lambda_min(K)|)' % (float(etas.min()), theta_min))


def quadrature(node_list, etas, fn, check=True):
    """Per-probe sums sum_i tau_i^2 fn(theta_i + eta) -> [nprobe, neta]."""
    etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
    if check:
        check_shifts(min_ritz(node_list), etas)
    if node_list and len({theta.size for theta, _ in node_list}) == 1:
        # every probe's rule has the same length (the rule): one array op over
        # [probe, eta, node]; the node sums run along the contiguous last axis as in
        # the per-probe form, so the values are the same bits (round 6: 0.38 -> 0.2 ms
        # of host time per cfg 5 step)
        th = numpy.stack([theta for theta, _ in node_list])
        w = numpy.stack([w for _, w in node_list])
        return numpy.sum(w[:, None, :] * fn(th[:, None, :] + etas[None, :, None]), axis=2)
    q = numpy.empty((len(node_list), etas.size))
    for p, (theta, w) in enumerate(node_list):   # all eta of a probe in one array op
        q[p] = numpy.sum(w[None, :] * fn(theta[None, :] + etas[:, None]), axis=1)
    return q


FUNCS = {
    'logdet': numpy.log,
    'traceinv': lambda x: 1.0 / x,
    'traceinv2': lambda x: 1.0 / (x * x),
}


def rademacher(n, num, seed, offset=0):
    """Rademacher probes (+-1), the counter-based generator of the device
    kernel: sign bit of splitmix64(seed * G + (offset + s) * H + i)."""
    i = numpy.arange(n, dtype=numpy.uint64)
    out = numpy.empty((n, num))
    with numpy.errstate(over='ignore'):
        for s in range(num):
            x = (numpy.uint64(seed) * numpy.uint64(0x9E3779B97F4A7C15) +
                 numpy.uint64(s + offset) * numpy.uint64(0xD1B54A32D192ED03) + i)
            x = x + numpy.uint64(0x9E3779B97F4A7C15)
            x = (x ^ (x >> numpy.uint64(30))) * numpy.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> numpy.uint64(27))) * numpy.uint64(0x94D049BB133111EB)
            x = x ^ (x >> numpy.uint64(31))
            out[:, s] = numpy.where((x >> numpy.uint64(63)) == 1, -1.0, 1.0)
    return out
