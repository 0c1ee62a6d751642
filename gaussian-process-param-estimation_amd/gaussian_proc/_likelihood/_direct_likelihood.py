"""Restricted GP log-likelihood in the direct parameters (sigma, sigma0).

Drop-in for ``DirectLikelihood`` of the reference
(gaussian_proc/_likelihood/_direct_likelihood.py:25-405).

Hot path. The reference evaluates one ``log_likelihood`` with
``K_mixed.logdet(eta)`` and two dense solves (:59, :62, :332), i.e. 2-3 dense
factorizations. Here, when ``K_mixed`` is the device operator, one Cholesky
K + eta I = L L^T gives everything: with R = [X | z] and
G = R^T (K + eta I)^-1 R = (L^-1 R)^T (L^-1 R),

  logdet_S = n log sigma^2 + logdet(K + eta I)              (:60)
  B        = X^T S^-1 X = G_XX / sigma^2                     (:65, :69)
  z^T M z  = (G_zz - G_Xz^T G_XX^-1 G_Xz) / sigma^2          (:71-72, :335-338)
  lp       = -(n-m)/2 log 2pi - logdet_S/2 - log det B / 2 - z^T M z / 2   (:75-76)

The sigma ~ 0 branch (|sigma| < 1e-8, :49-55) never touches K and is evaluated
as in the reference. The Jacobian / Hessian keep the reference formulas
(derivatives w.r.t. sigma^2 and sigma0^2 — reference quirk) on top
of the operator duck type; on the dense eigenvalue operator (sigma not ~ 0) the
same quantities come from the band Gram blocks Gp = R^T (K + eta I)^-p R,
p = 1..3, and tr((K + eta I)^-1), tr((K + eta I)^-2) from the same factor
(selected inversion and its eta-tangent; _jac_hess_from_terms), with no dense
solve and no eigenvalues.
"""

import numpy
import scipy.optimize
from functools import partial

from ._profile_likelihood import _use_band

__all__ = ['DirectLikelihood']

_TOL = 1e-8          # _direct_likelihood.py:49,106,324
_TOL_HESS = 1e-16    # _direct_likelihood.py:179
_CANCEL = 1e-4       # band-path derivative forms: least kept fraction (_jac_hess_from_terms)


def _lp_from_terms(n, m, sigma, logdet_kn, G):
    """log-likelihood from logdet(K + eta I) and G = R^T (K + eta I)^-1 R."""
    s2 = sigma ** 2
    Gxx = G[:m, :m]
    gxz = G[:m, m]
    gzz = G[m, m]
    logdet_S = n * numpy.log(s2) + logdet_kn
    B = Gxx / s2
    logdet_B = numpy.log(numpy.linalg.det(B))
    zMz = (gzz - gxz @ numpy.linalg.solve(Gxx, gxz)) / s2
    return -0.5 * (n - m) * numpy.log(2.0 * numpy.pi) - 0.5 * logdet_S \
        - 0.5 * logdet_B - 0.5 * zMz


def _lp_from_terms_batch(n, m, sigma, logdet_kn, G):
    """_lp_from_terms for a batch: logdet_kn [E], G [E, m+1, m+1] -> lp [E] (the
    same formula with numpy's stacked det / solve: one call per step of a sweep
    instead of E)."""
    G = numpy.asarray(G, dtype=float)
    s2 = sigma ** 2
    Gxx = G[:, :m, :m]
    gxz = G[:, :m, m]
    gzz = G[:, m, m]
    logdet_S = n * numpy.log(s2) + numpy.asarray(logdet_kn, dtype=float)
    logdet_B = numpy.log(numpy.linalg.det(Gxx / s2))
    zMz = (gzz - numpy.einsum('ei,ei->e', gxz,
                              numpy.linalg.solve(Gxx, gxz[:, :, None])[:, :, 0])) / s2
    return -0.5 * (n - m) * numpy.log(2.0 * numpy.pi) - 0.5 * logdet_S \
        - 0.5 * logdet_B - 0.5 * zMz


def _lp_small_sigma(z, X, sigma0):
    """|sigma| < tol branch (_direct_likelihood.py:50-55, M_dot :325-328)."""
    n, m = X.shape
    s02 = sigma0 ** 2
    logdet_S = n * numpy.log(s02)
    Y = X / s02
    B = X.T @ Y
    logdet_B = numpy.log(numpy.linalg.det(B))
    Binv = numpy.linalg.inv(B)
    Mz = z / s02 - Y @ (Binv @ (Y.T @ z))
    return -0.5 * (n - m) * numpy.log(2.0 * numpy.pi) - 0.5 * logdet_S \
        - 0.5 * logdet_B - 0.5 * numpy.dot(z, Mz)


def _jac_hess_from_terms(n, m, sigma, eta, G1, G2, G3, tr1, tr2=None):
    """Jacobian (and Hessian when tr2 = tr((K + eta I)^-2) is given) of the
    direct likelihood for |sigma| >= tol from Gp = R^T A^-p R, A = K + eta I,
    S = sigma^2 A. With a = G1_XX^-1 G1_Xz and r = z - X a (so X^T A^-1 r = 0):
    M z = A^-1 r / sigma^2, K M z = (r - eta A^-1 r) / sigma^2, and every term of
    _direct_likelihood.py:89-270 is a quadratic form Qp = r^T A^-p r or uses
    t2 = X^T A^-2 r, c = G1_XX^-1 t2.

    The reference forms K M z as a product with K; here it is r - eta A^-1 r, so
    the K-weighted forms are differences such as Q1 - eta Q2. When eta is large
    against the spectrum carrying r they cancel: if a difference keeps less than
    _CANCEL of its largest term, this returns None and the caller takes the
    reference's solve path."""
    s2 = sigma ** 2
    Gxx = G1[:m, :m]
    a = numpy.linalg.solve(Gxx, G1[:m, m])

    def quad(G):
        return G[m, m] - 2.0 * (a @ G[:m, m]) + a @ G[:m, :m] @ a

    def kept(total, *terms):
        return abs(total) >= _CANCEL * max(abs(t) for t in terms)

    Q1, Q2 = quad(G1), quad(G2)
    P2 = numpy.linalg.solve(Gxx, G2[:m, :m])          # G1_XX^-1 G2_XX
    trace_M = (tr1 - numpy.trace(P2)) / s2
    trace_KM = (n - m) / s2 - eta * trace_M
    zMMz = Q2 / s2 ** 2
    zMKMz = (Q1 - eta * Q2) / s2 ** 2
    if not kept(Q1 - eta * Q2, Q1, eta * Q2):
        return None, None
    jac = numpy.array([-0.5 * trace_KM + 0.5 * zMKMz, -0.5 * trace_M + 0.5 * zMMz], dtype=float)
    if tr2 is None:
        return jac, None
    Q3 = quad(G3)
    t2 = G2[:m, m] - G2[:m, :m] @ a
    tc = t2 @ numpy.linalg.solve(Gxx, t2)             # t2^T c
    zMMMz = (Q3 - tc) / s2 ** 3
    zMMKMz = (Q2 - eta * Q3 + eta * tc) / s2 ** 3
    zMKMKMz = (Q1 - 2.0 * eta * Q2 + eta ** 2 * (Q3 - tc)) / s2 ** 3
    if not (kept(Q2 - eta * Q3 + eta * tc, Q2, eta * Q3, eta * tc) and
            kept(Q1 - 2.0 * eta * Q2 + eta ** 2 * (Q3 - tc), Q1, 2.0 * eta * Q2, eta ** 2 * Q3,
                 eta ** 2 * tc)):
        return jac, None
    trace_M2 = (tr2 - 2.0 * numpy.trace(numpy.linalg.solve(Gxx, G3[:m, :m])) +
                numpy.trace(P2 @ P2)) / s2 ** 2
    trace_KMKM = (n - m) / s2 ** 2 - (2 * eta / s2) * trace_M + (eta ** 2) * trace_M2
    trace_KMM = trace_M / s2 - eta * trace_M2
    h_ss = 0.5 * (trace_KMKM - 2.0 * zMKMKMz)
    h_s0 = 0.5 * (trace_KMM - 2.0 * zMMKMz)
    h_00 = 0.5 * (trace_M2 - 2.0 * zMMMz)
    return jac, numpy.array([[h_ss, h_s0], [h_s0, h_00]], dtype=float)


class DirectLikelihood(object):

    @staticmethod
    def log_likelihood(z, X, K_mixed, sign_switch, hyperparam):
        sigma, sigma0 = hyperparam[0], hyperparam[1]
        n, m = X.shape
        if numpy.abs(sigma) < _TOL:
            lp = _lp_small_sigma(z, X, sigma0)
        elif hasattr(K_mixed, 'loglik_terms'):
            eta = (sigma0 / sigma) ** 2
            ld, G = K_mixed.loglik_terms([eta], X, z)
            lp = _lp_from_terms(n, m, sigma, ld[0], G[0])
        else:
            # generic operator duck type (reference call pattern)
            eta = (sigma0 / sigma) ** 2
            logdet_S = n * numpy.log(sigma ** 2) + K_mixed.logdet(eta)
            Y = K_mixed.solve(eta, X) / sigma ** 2
            B = X.T @ Y
            logdet_B = numpy.log(numpy.linalg.det(B))
            Binv = numpy.linalg.inv(B)
            zMz = numpy.dot(z, DirectLikelihood.M_dot(K_mixed, Binv, Y, sigma, sigma0, z))
            lp = -0.5 * (n - m) * numpy.log(2.0 * numpy.pi) - 0.5 * logdet_S \
                - 0.5 * logdet_B - 0.5 * zMz
        return -lp if sign_switch else lp

    @staticmethod
    def log_likelihood_batch(z, X, K_mixed, hyperparams, sign_switch=False):
        """Vectorised log_likelihood over many (sigma, sigma0): all etas are
        factorized in batches of ``K_mixed.op.max_batch`` per device call."""
        hp = numpy.atleast_2d(numpy.asarray(hyperparams, dtype=float))
        n, m = X.shape
        out = numpy.empty(hp.shape[0])
        big = numpy.abs(hp[:, 0]) >= _TOL
        if numpy.any(big):
            etas = (hp[big, 1] / hp[big, 0]) ** 2
            ld, G = K_mixed.loglik_terms(etas, X, z)
            out[big] = [_lp_from_terms(n, m, s, l, g)
                        for s, l, g in zip(hp[big, 0], ld, G)]
        for i in numpy.flatnonzero(~big):
            out[i] = _lp_small_sigma(z, X, hp[i, 1])
        return -out if sign_switch else out

    @staticmethod
    def M_dot(K_mixed, Binv, Y, sigma, sigma0, z):                 # :276-340
        if numpy.abs(sigma) < _TOL:
            w = z / sigma0 ** 2
        else:
            eta = (sigma0 / sigma) ** 2
            w = K_mixed.solve(eta, z) / sigma ** 2
        return w - Y @ (Binv @ (Y.T @ z))

    @staticmethod
    def log_likelihood_jacobian(z, X, K_mixed, sign_switch, hyperparam):   # :89-157
        sigma, sigma0 = hyperparam[0], hyperparam[1]
        n, m = X.shape
        small = numpy.abs(sigma) < _TOL
        if not small and _use_band(K_mixed):
            eta = (sigma0 / sigma) ** 2
            # traceinv=2: tr((K + eta I)^-2) rides on the same call (+1.5 ms at N = 16384)
            # so that the Hessian at this point, which trust-exact (the reference's
            # optimizer, :378) evaluates at every iterate after the Jacobian, comes from
            # the operator's cache instead of a second factorization (+2.7 ms)
            _, G1, G2, G3, tr1, _ = K_mixed.der_terms([eta], X, z, traceinv=2)
            jac = _jac_hess_from_terms(n, m, sigma, eta, G1[0], G2[0], G3[0], tr1[0])[0]
            if jac is not None:
                return -jac if sign_switch else jac
        if small:
            Y = X / sigma0 ** 2
        else:
            eta = (sigma0 / sigma) ** 2
            Y = K_mixed.solve(eta, X) / sigma ** 2
        Binv = numpy.linalg.inv(X.T @ Y)
        Mz = DirectLikelihood.M_dot(K_mixed, Binv, Y, sigma, sigma0, z)
        KMz = K_mixed.dot(0, Mz)
        zMMz = numpy.dot(Mz, Mz)
        zMKMz = numpy.dot(Mz, KMz)
        if small:
            trace_M = (n - m) / sigma0 ** 2
            YtKY = Y.T @ K_mixed.dot(0, Y)
            trace_KM = K_mixed.trace(0) / sigma0 ** 2 - numpy.trace(Binv @ YtKY)
        else:
            trace_M = K_mixed.traceinv(eta) / sigma ** 2 - numpy.trace(Binv @ (Y.T @ Y))
            trace_KM = (n - m) / sigma ** 2 - eta * trace_M
        jac = numpy.array([-0.5 * trace_KM + 0.5 * zMKMz,
                           -0.5 * trace_M + 0.5 * zMMz], dtype=float)
        return -jac if sign_switch else jac

    @staticmethod
    def log_likelihood_hessian(z, X, K_mixed, sign_switch, hyperparam):    # :163-270
        sigma, sigma0 = hyperparam[0], hyperparam[1]
        n, m = X.shape
        small = numpy.abs(sigma) < _TOL_HESS
        if not small and _use_band(K_mixed):
            eta = (sigma0 / sigma) ** 2
            _, G1, G2, G3, tr1, tr2 = K_mixed.der_terms([eta], X, z, traceinv=2)
            hess = _jac_hess_from_terms(n, m, sigma, eta, G1[0], G2[0], G3[0], tr1[0],
                                        tr2[0])[1]
            if hess is not None:
                return -hess if sign_switch else hess
        if small:
            Y = X / sigma0 ** 2
            V = Y / sigma0 ** 2
        else:
            eta = (sigma0 / sigma) ** 2
            Y = K_mixed.solve(eta, X) / sigma ** 2
            V = K_mixed.solve(eta, Y) / sigma ** 2
        Binv = numpy.linalg.inv(X.T @ Y)
        A = Binv @ (Y.T @ Y)
        Mz = DirectLikelihood.M_dot(K_mixed, Binv, Y, sigma, sigma0, z)
        MMz = DirectLikelihood.M_dot(K_mixed, Binv, Y, sigma, sigma0, Mz)
        KMz = K_mixed.dot(0, Mz)
        MKMz = DirectLikelihood.M_dot(K_mixed, Binv, Y, sigma, sigma0, KMz)
        zMMMz = numpy.dot(Mz, MMz)
        zMMKMz = numpy.dot(MMz, KMz)
        zMKMKMz = numpy.dot(KMz, MKMz)
        if small:
            trace_M = (n - m) / sigma0 ** 2
            trace_S2inv = n / sigma0 ** 4
        else:
            trace_M = K_mixed.traceinv(eta) / sigma ** 2 - numpy.trace(A)
            trace_S2inv = K_mixed.traceinv(eta, exponent=2) / sigma ** 4
        trace_M2 = trace_S2inv - 2.0 * numpy.trace(Binv @ (Y.T @ V)) + numpy.trace(A @ A)
        if small:
            E = K_mixed.dot(0, X, exponent=2) @ (X.T @ X)
            trace_KMKM = (K_mixed.trace(0, exponent=2) - 2.0 * numpy.trace(E) +
                          numpy.trace(E @ E)) / sigma0 ** 4
            YtKY = Y.T @ K_mixed.dot(0, Y)
            trace_KM = K_mixed.trace(0) / sigma0 ** 2 - numpy.trace(Binv @ YtKY)
            trace_KMM = trace_KM / sigma0 ** 2
        else:
            trace_KMKM = (n - m) / sigma ** 4 - (2 * eta / sigma ** 2) * trace_M + \
                (eta ** 2) * trace_M2
            trace_KMM = trace_M / sigma ** 2 - eta * trace_M2
        h_ss = 0.5 * (trace_KMKM - 2.0 * zMKMKMz)
        h_s0 = 0.5 * (trace_KMM - 2.0 * zMMKMz)
        h_00 = 0.5 * (trace_M2 - 2.0 * zMMMz)
        hess = numpy.array([[h_ss, h_s0], [h_s0, h_00]], dtype=float)
        return -hess if sign_switch else hess

    @staticmethod
    def maximize_log_likelihood(z, X, K_mixed, tol=1e-3, hyperparam_guess=[0.2, 0.2],
                                method='Nelder-Mead'):                      # :346-405
        print('Maximize log likelihood with sigma sigma0 ...')
        f = partial(DirectLikelihood.log_likelihood, z, X, K_mixed, True)
        jac = partial(DirectLikelihood.log_likelihood_jacobian, z, X, K_mixed, True)
        hess = partial(DirectLikelihood.log_likelihood_hessian, z, X, K_mixed, True)
        # The reference overrides ``method`` with trust-exact (:378).
        res = scipy.optimize.minimize(f, hyperparam_guess, method='trust-exact', tol=tol,
                                      jac=jac, hess=hess)
        print(res)
        print('Iter: %d, Eval: %d, Success: %s' % (res.nit, res.nfev, res.success))
        sigma, sigma0 = res.x[0], res.x[1]
        return {'sigma': sigma, 'sigma0': sigma0, 'eta': (sigma0 / sigma) ** 2,
                'max_lp': -res.fun}
