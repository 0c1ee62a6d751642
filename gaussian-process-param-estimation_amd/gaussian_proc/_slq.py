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


def nodes(alpha, beta):
    """Ritz values and squared first components for each probe.
    alpha, beta: [nprobe, steps]; beta[p, k] = 0 ends probe p's tridiagonal
    after step k."""
    out = []
    for a, b in zip(alpha, beta):
        k = len(a)
        z = numpy.flatnonzero(b == 0.0)
        if z.size:
            k = int(z[0]) + 1
        T = numpy.diag(a[:k]) + numpy.diag(b[:k - 1], 1) + numpy.diag(b[:k - 1], -1)
        theta, U = numpy.linalg.eigh(T)
        out.append((theta, U[0] ** 2))
    return out


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
