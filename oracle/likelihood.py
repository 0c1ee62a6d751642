"""Direct and profiled GP log-likelihood (oracle restatement; TEST
INFRASTRUCTURE ONLY).

Restates, operator-agnostic (``op`` is any object with the MixedCorrelation
duck type: logdet / traceinv / trace / solve / dot):

  direct_lp        _direct_likelihood.py:31-83  (restricted likelihood in (sigma, sigma0))
  direct_jac       _direct_likelihood.py:89-157 (derivatives w.r.t. sigma^2, sigma0^2 —
                                                 reference quirk, SURVEY §0.4, kept)
  direct_hess      _direct_likelihood.py:163-270
  m_dot            _direct_likelihood.py:276-340
  profile_lp       _profile_likelihood.py:38-85
  profile_der1_eta _profile_likelihood.py:91-132
  profile_der2_eta _profile_likelihood.py:138-192

Thresholds are the reference's: 1e-8 for lp/jac/M_dot, 1e-16 for the Hessian.
"""

import numpy

TOL_LP = 1e-8        # _direct_likelihood.py:49,106,324
TOL_HESS = 1e-16     # _direct_likelihood.py:179


def _sinv_x(op, X, sigma, sigma0, tol):
    """Y = S^-1 X with S = sigma^2 K + sigma0^2 I (via K + eta I)."""
    if abs(sigma) < tol:
        return X / sigma0 ** 2
    eta = (sigma0 / sigma) ** 2
    return op.solve(eta, X) / sigma ** 2


def m_dot(op, Binv, Y, sigma, sigma0, z):
    """M z = S^-1 z - Y B^-1 Y^T z   (_direct_likelihood.py:323-340)."""
    w = _sinv_x(op, z, sigma, sigma0, TOL_LP)
    return w - Y @ (Binv @ (Y.T @ z))


def direct_lp(z, X, op, hyperparam, sign_switch=False):
    sigma, sigma0 = hyperparam[0], hyperparam[1]
    n, m = X.shape
    if abs(sigma) < TOL_LP:
        logdet_S = n * numpy.log(sigma0 ** 2)
        Y = X / sigma0 ** 2
    else:
        eta = (sigma0 / sigma) ** 2
        logdet_S = n * numpy.log(sigma ** 2) + op.logdet(eta)
        Y = op.solve(eta, X) / sigma ** 2
    B = X.T @ Y
    logdet_B = numpy.log(numpy.linalg.det(B))
    Binv = numpy.linalg.inv(B)
    zMz = numpy.dot(z, m_dot(op, Binv, Y, sigma, sigma0, z))
    lp = -0.5 * (n - m) * numpy.log(2.0 * numpy.pi) - 0.5 * logdet_S \
        - 0.5 * logdet_B - 0.5 * zMz
    return -lp if sign_switch else lp


def direct_jac(z, X, op, hyperparam, sign_switch=False):
    sigma, sigma0 = hyperparam[0], hyperparam[1]
    n, m = X.shape
    small = abs(sigma) < TOL_LP
    Y = _sinv_x(op, X, sigma, sigma0, TOL_LP)
    B = X.T @ Y
    Binv = numpy.linalg.inv(B)
    Mz = m_dot(op, Binv, Y, sigma, sigma0, z)
    KMz = op.dot(0, Mz)
    zMMz = numpy.dot(Mz, Mz)
    zMKMz = numpy.dot(Mz, KMz)
    if small:
        trace_M = (n - m) / sigma0 ** 2
        YtKY = Y.T @ op.dot(0, Y)
        trace_KM = op.trace(0) / sigma0 ** 2 - numpy.trace(Binv @ YtKY)
    else:
        eta = (sigma0 / sigma) ** 2
        trace_M = op.traceinv(eta) / sigma ** 2 - numpy.trace(Binv @ (Y.T @ Y))
        trace_KM = (n - m) / sigma ** 2 - eta * trace_M
    jac = numpy.array([-0.5 * trace_KM + 0.5 * zMKMz,
                       -0.5 * trace_M + 0.5 * zMMz], dtype=float)
    return -jac if sign_switch else jac


def direct_hess(z, X, op, hyperparam, sign_switch=False):
    sigma, sigma0 = hyperparam[0], hyperparam[1]
    n, m = X.shape
    small = abs(sigma) < TOL_HESS
    if small:
        Y = X / sigma0 ** 2
        V = Y / sigma0 ** 2
    else:
        eta = (sigma0 / sigma) ** 2
        Y = op.solve(eta, X) / sigma ** 2
        V = op.solve(eta, Y) / sigma ** 2
    B = X.T @ Y
    Binv = numpy.linalg.inv(B)
    A = Binv @ (Y.T @ Y)
    Mz = m_dot(op, Binv, Y, sigma, sigma0, z)
    MMz = m_dot(op, Binv, Y, sigma, sigma0, Mz)
    KMz = op.dot(0, Mz)
    zMMMz = numpy.dot(Mz, MMz)
    MKMz = m_dot(op, Binv, Y, sigma, sigma0, KMz)
    zMMKMz = numpy.dot(MMz, KMz)
    zMKMKMz = numpy.dot(KMz, MKMz)
    if small:
        trace_M = (n - m) / sigma0 ** 2
        trace_S2inv = n / sigma0 ** 4
    else:
        trace_M = op.traceinv(eta) / sigma ** 2 - numpy.trace(A)
        trace_S2inv = op.traceinv(eta, exponent=2) / sigma ** 4
    trace_M2 = trace_S2inv - 2.0 * numpy.trace(Binv @ (Y.T @ V)) + \
        numpy.trace(A @ A)
    if small:
        D = X.T @ X
        E = op.dot(0, X, exponent=2) @ D
        trace_KMKM = (op.trace(0, exponent=2) - 2.0 * numpy.trace(E) +
                      numpy.trace(E @ E)) / sigma0 ** 4
        YtKY = Y.T @ op.dot(0, Y)
        trace_KM = op.trace(0) / sigma0 ** 2 - numpy.trace(Binv @ YtKY)
        trace_KMM = trace_KM / sigma0 ** 2
    else:
        trace_KMKM = (n - m) / sigma ** 4 - (2 * eta / sigma ** 2) * trace_M + \
            (eta ** 2) * trace_M2
        trace_KMM = trace_M / sigma ** 2 - eta * trace_M2
    d00 = 0.5 * (trace_KMKM - 2.0 * zMKMKMz)
    d01 = 0.5 * (trace_KMM - 2.0 * zMMKMz)
    d11 = 0.5 * (trace_M2 - 2.0 * zMMMz)
    hess = numpy.array([[d00, d01], [d01, d11]], dtype=float)
    return -hess if sign_switch else hess


def profile_lp(z, X, op, hyperparam, sign_switch=False):
    """_profile_likelihood.py:57-85. The reference materialises Y B^-1 Y^T
    (n x n, :73); the same value is computed here in O(nm)."""
    sigma, eta = hyperparam[0], hyperparam[1]
    n, m = X.shape
    logdet_Kn = op.logdet(eta)
    Y = op.solve(eta, X)
    w = op.solve(eta, z)
    B = X.T @ Y
    logdet_B = numpy.log(numpy.linalg.det(B))
    Binv = numpy.linalg.inv(B)
    zMz = numpy.dot(z, w - Y @ (Binv @ (Y.T @ z)))
    lp = -0.5 * (n - m) * numpy.log(sigma ** 2) - 0.5 * logdet_Kn \
        - 0.5 * logdet_B - (0.5 / (sigma ** 2)) * zMz
    return -lp if sign_switch else lp


def profile_der1_eta(z, X, op, log_eta):
    """_profile_likelihood.py:98-132."""
    eta = 0.0 if numpy.isneginf(log_eta) else 10.0 ** log_eta
    Y = op.solve(eta, X)
    w = op.solve(eta, z)
    n, m = X.shape
    B = X.T @ Y
    Binv = numpy.linalg.inv(B)
    Mz = w - Y @ (Binv @ (Y.T @ z))
    trace_M = op.traceinv(eta) - numpy.trace(Binv @ (Y.T @ Y))
    zMz = numpy.dot(z, Mz)
    zM2z = numpy.dot(Mz, Mz)
    sigma02 = zMz / (n - m)
    return -0.5 * (trace_M - zM2z / sigma02)


def profile_der2_eta(z, X, op, eta):
    """_profile_likelihood.py:146-192."""
    Y = op.solve(eta, X)
    V = op.solve(eta, Y)
    w = op.solve(eta, z)
    n, m = X.shape
    B = X.T @ Y
    Binv = numpy.linalg.inv(B)
    Mz = w - Y @ (Binv @ (Y.T @ z))
    A = Binv @ (Y.T @ Y)
    trace_M = op.traceinv(eta) - numpy.trace(A)
    trace_M2 = op.traceinv(eta, exponent=2) - \
        2.0 * numpy.trace(Binv @ (Y.T @ V)) + numpy.trace(A @ A)
    MMz = op.solve(eta, Mz) - Y @ (Binv @ (Y.T @ Mz))
    zMz = numpy.dot(z, Mz)
    zM3z = numpy.dot(Mz, MMz)
    sigma02 = zMz / (n - m)
    return (0.5 / sigma02) * ((trace_M2 / (n - m) + (trace_M / (n - m)) ** 2) *
                              zMz - 2.0 * zM3z)
