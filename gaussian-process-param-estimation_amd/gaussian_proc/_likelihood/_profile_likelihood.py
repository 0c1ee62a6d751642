"""Profiled GP log-likelihood in (sigma, eta).

Drop-in for ``ProfileLikelihood`` of the reference
(gaussian_proc/_likelihood/_profile_likelihood.py:32-415).

``log_likelihood`` (:38-85) uses the same single-factorization terms as the
direct likelihood: with G = [X z]^T (K + eta I)^-1 [X z],
  lp = -(n-m)/2 log sigma^2 - logdet(K + eta I)/2 - log det G_XX / 2
       - (G_zz - G_Xz^T G_XX^-1 G_Xz) / (2 sigma^2).
The reference materialises Y B^-1 Y^T as an n x n matrix (:73); the value is the
same. The eta-derivatives (:91-192) keep the reference formulas on the operator
duck type; on the dense eigenvalue operator they come instead from the Gram
blocks Gp = [X z]^T (K + eta I)^-p [X z], p = 1..3, of the band path
(MixedCorrelation.der_terms, any number of eta per call) and traceinv of
exponents 1 and 2 from the same factor (selected inversion and its eta-tangent),
with the same algebra written in those blocks (_der_from_terms).
"""

import numpy
from scipy.optimize import minimize
from functools import partial

from ._root_finding import chandrupatla_method, BatchedFunction, \
    find_interval_with_sign_change_batched

__all__ = ['ProfileLikelihood']


def _use_band(K_mixed):
    return hasattr(K_mixed, 'der_terms') and getattr(K_mixed, 'imate_method', None) == \
        'eigenvalue'


def _der_from_terms(n, m, G1, G2, G3, tr1, tr2=None):
    """der1 (and der2 when tr2 is given) of the profiled likelihood from
    Gp = [X z]^T S^-p [X z], S = K + eta I, and tr(S^-1), tr(S^-2); the terms of
    _profile_likelihood.py:91-192 in those blocks: Mz = S^-1 (z - X a) with
    a = B^-1 X^T S^-1 z, B = X^T S^-1 X."""
    B = G1[:m, :m]
    a = numpy.linalg.solve(B, G1[:m, m])
    zMz = G1[m, m] - G1[:m, m] @ a
    zM2z = G2[m, m] - 2.0 * (a @ G2[:m, m]) + a @ G2[:m, :m] @ a
    A = numpy.linalg.solve(B, G2[:m, :m])            # B^-1 Y^T Y
    trace_M = tr1 - numpy.trace(A)
    sigma02 = zMz / (n - m)
    der1 = -0.5 * (trace_M - zM2z / sigma02)
    if tr2 is None:
        return der1, None
    trace_M2 = tr2 - 2.0 * numpy.trace(numpy.linalg.solve(B, G3[:m, :m])) + numpy.trace(A @ A)
    MzS1Mz = G3[m, m] - 2.0 * (a @ G3[:m, m]) + a @ G3[:m, :m] @ a
    YtMz = G2[:m, m] - G2[:m, :m] @ a
    zM3z = MzS1Mz - YtMz @ numpy.linalg.solve(B, YtMz)
    der2 = (0.5 / sigma02) * ((trace_M2 / (n - m) + (trace_M / (n - m)) ** 2) * zMz -
                              2.0 * zM3z)
    return der1, der2


class ProfileLikelihood(object):

    @staticmethod
    def log_likelihood(z, X, K_mixed, sign_switch, hyperparam):
        sigma, eta = hyperparam[0], hyperparam[1]
        n, m = X.shape
        if hasattr(K_mixed, 'loglik_terms'):
            ld, G = K_mixed.loglik_terms([eta], X, z)
            ld, G = ld[0], G[0]
            Gxx, gxz, gzz = G[:m, :m], G[:m, m], G[m, m]
            logdet_B = numpy.log(numpy.linalg.det(Gxx))
            zMz = gzz - gxz @ numpy.linalg.solve(Gxx, gxz)
        else:
            ld = K_mixed.logdet(eta)
            Y = K_mixed.solve(eta, X)
            w = K_mixed.solve(eta, z)
            B = X.T @ Y
            logdet_B = numpy.log(numpy.linalg.det(B))
            zMz = numpy.dot(z, w - Y @ (numpy.linalg.inv(B) @ (Y.T @ z)))
        lp = -0.5 * (n - m) * numpy.log(sigma ** 2) - 0.5 * ld - 0.5 * logdet_B \
            - (0.5 / (sigma ** 2)) * zMz
        return -lp if sign_switch else lp

    @staticmethod
    def _mz(z, X, K_mixed, eta):
        Y = K_mixed.solve(eta, X)
        w = K_mixed.solve(eta, z)
        Binv = numpy.linalg.inv(X.T @ Y)
        return Y, Binv, w - Y @ (Binv @ (Y.T @ z))

    @staticmethod
    def log_likelihood_der1_eta(z, X, K_mixed, log_eta):           # :91-132
        eta = 0.0 if numpy.isneginf(log_eta) else 10.0 ** log_eta
        n, m = X.shape
        if _use_band(K_mixed):
            return float(ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, K_mixed,
                                                                         [log_eta])[0])
        Y, Binv, Mz = ProfileLikelihood._mz(z, X, K_mixed, eta)
        trace_M = K_mixed.traceinv(eta) - numpy.trace(Binv @ (Y.T @ Y))
        zMz = numpy.dot(z, Mz)
        zM2z = numpy.dot(Mz, Mz)
        sigma02 = zMz / (n - m)
        return -0.5 * (trace_M - zM2z / sigma02)

    @staticmethod
    def log_likelihood_der1_eta_batch(z, X, K_mixed, log_etas):
        """der1 at many log10(eta) in one device call (dense eigenvalue
        operator; otherwise one log_likelihood_der1_eta per point)."""
        log_etas = numpy.atleast_1d(numpy.asarray(log_etas, dtype=float))
        if not _use_band(K_mixed):
            return numpy.array([ProfileLikelihood.log_likelihood_der1_eta(z, X, K_mixed, le)
                                for le in log_etas])
        n, m = X.shape
        etas = numpy.where(numpy.isneginf(log_etas), 0.0, 10.0 ** log_etas)
        _, G1, G2, G3, tr1 = K_mixed.der_terms(etas, X, z, traceinv=True)
        return numpy.array([_der_from_terms(n, m, G1[i], G2[i], G3[i], tr1[i])[0]
                            for i in range(etas.size)])

    @staticmethod
    def log_likelihood_der2_eta(z, X, K_mixed, eta):               # :138-192
        n, m = X.shape
        if _use_band(K_mixed):
            _, G1, G2, G3, tr1, tr2 = K_mixed.der_terms([eta], X, z, traceinv=2)
            return float(_der_from_terms(n, m, G1[0], G2[0], G3[0], tr1[0], tr2[0])[1])
        Y, Binv, Mz = ProfileLikelihood._mz(z, X, K_mixed, eta)
        V = K_mixed.solve(eta, Y)
        A = Binv @ (Y.T @ Y)
        trace_M = K_mixed.traceinv(eta) - numpy.trace(A)
        trace_M2 = K_mixed.traceinv(eta, exponent=2) - \
            2.0 * numpy.trace(Binv @ (Y.T @ V)) + numpy.trace(A @ A)
        MMz = K_mixed.solve(eta, Mz) - Y @ (Binv @ (Y.T @ Mz))
        zMz = numpy.dot(z, Mz)
        zM3z = numpy.dot(Mz, MMz)
        sigma02 = zMz / (n - m)
        return (0.5 / sigma02) * ((trace_M2 / (n - m) + (trace_M / (n - m)) ** 2) * zMz -
                                  2.0 * zM3z)

    @staticmethod
    def maximize_log_likelihood_with_sigma_eta(z, X, K_mixed, tol=1e-6,
                                               hyperparam_guess=[0.1, 0.1],
                                               method='Nelder-Mead'):   # :198-238
        print('Maximize log likelihood with sigma eta ...')
        f = partial(ProfileLikelihood.log_likelihood, z, X, K_mixed, True)
        res = minimize(f, hyperparam_guess, method='Nelder-Mead', tol=tol)
        print('Iter: %d, Eval: %d, success: %s' % (res.nit, res.nfev, res.success))
        sigma, eta = res.x[0], res.x[1]
        return {'sigma': sigma, 'sigma0': numpy.sqrt(eta) * sigma, 'eta': eta,
                'max_lp': -res.fun}

    @staticmethod
    def find_log_likelihood_der1_zeros(z, X, K_mixed, interval_eta, tol=1e-6,
                                       max_iterations=100, num_bracket_trials=3,
                                       group=False, speculative=None):  # :244-415
        """Root of d lp / d eta in log10(eta) (reference :244-415: bracket search,
        then Chandrupatla, then the optimal sigma). The der1 evaluations are
        batched: the bracket search requests every point it may need next in one
        call (_root_finding.find_interval_with_sign_change_batched), sharded over
        the ranks of a torch.distributed ``group`` when the caller passes one
        (sweep.der1_sweep: one all-gather per batch; every rank must hold the
        same K, X, z, so sharding is opt-in: the default False keeps the search
        on the local device). Chandrupatla's iterations are speculative: each
        device call also evaluates up to ``speculative`` points the next
        iterations may need (_root_finding._chandrupatla_candidates; default 64
        on the band operator, where a batch of eta costs one banded Cholesky's
        latency, else 0). Decisions and results are those of the sequential
        reference driver."""
        n, m = X.shape

        def optimal_sigma(eta):
            if hasattr(K_mixed, 'loglik_terms') and eta > 0:
                _, G = K_mixed.loglik_terms([eta], X, z)
                G = G[0]
                zMz = G[m, m] - G[:m, m] @ numpy.linalg.solve(G[:m, :m], G[:m, m])
                return numpy.sqrt(zMz / (n - m))
            Y, Binv, Mz = ProfileLikelihood._mz(z, X, K_mixed, eta)
            return numpy.sqrt(numpy.dot(z, Mz) / (n - m))

        def optimal_sigma0():
            Binv = numpy.linalg.inv(X.T @ X)
            v = X @ (Binv @ (X.T @ z))
            return numpy.sqrt(numpy.dot(z, z - v) / (n - m))

        from ..sweep import der1_sweep
        if speculative is None:
            speculative = 64 if _use_band(K_mixed) else 0
        fb = BatchedFunction(lambda le: der1_sweep(K_mixed, X, z, le, group=group),
                             spec_budget=speculative)
        print('Find root of log likelihood derivative ...')
        bracket = [numpy.log10(interval_eta[0]), numpy.log10(interval_eta[1])]
        found, bracket, values = find_interval_with_sign_change_batched(
            fb, bracket, num_bracket_trials, tol=tol)
        if found:
            res = chandrupatla_method(fb, bracket, values, verbose=False, eps_m=tol,
                                      eps_a=tol, maxiter=max_iterations)
            print('Iter: %d' % (res['iterations']))
            eta = 10 ** res['root']
            sigma = optimal_sigma(eta)
            sigma0 = numpy.sqrt(eta) * sigma
            success = True
        else:
            d2 = ProfileLikelihood.log_likelihood_der2_eta(z, X, K_mixed, 0.0)
            left, right = values[0], values[1]
            print('dL/deta   at eta = %0.2e:\t %0.2f' % (bracket[0], left))
            print('dL/deta   at eta = %0.2e:\t %0.16f' % (bracket[1], right))
            print('d2L/deta2 at eta = 0.0:\t %0.2f' % d2)
            eta = None
            if left > 0 and right > 0:
                eta = 0.0 if d2 > 0 else numpy.inf
            elif left < 0 and right < 0:
                eta = 0.0 if d2 < 0 else numpy.inf
            if eta == 0:
                sigma0 = 0
                sigma = optimal_sigma(eta)
            elif eta == numpy.inf:
                sigma = 0
                sigma0 = optimal_sigma0()
            else:
                raise ValueError('eta must be zero or inf at this point.')
            success = True
        ProfileLikelihood.last_der1_calls = (fb.calls, fb.points, dict(fb.memo))
        # the largest eta batch of one device call (<= 64: the band operator's
        # cyclic-reduction path, gpmi_band_der_terms)
        ProfileLikelihood.last_der1_max_batch = fb.max_points
        return {'sigma': sigma, 'sigma0': sigma0, 'eta': eta, 'success': success}
