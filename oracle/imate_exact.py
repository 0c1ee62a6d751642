"""Exact methods of the third-party ``imate`` package (oracle restatement;
TEST INFRASTRUCTURE ONLY).

``imate`` is listed unpinned in /root/reference/requirements.txt:5 and is absent
from this image (no network). The reference calls it through the 2021 API
(tuple returns ``(value, info)``, ``exponent=`` keyword) at
gaussian_proc/_mixed_correlation/mixed_correlation.py:44,65-66,109-143,178-209,245-268.
Only the *exact* methods are restated here, from their published definitions:

* ``logdet(A, method='eigenvalue', eigenvalues=lam, exponent=p)`` = p * sum(log lam)
* ``logdet(A, method='cholesky', exponent=p)`` = p * 2 * sum(log diag chol(A))
* ``traceinv(A, method='eigenvalue', eigenvalues=lam, exponent=p)`` = sum(lam^-p)
* ``traceinv(A, method='cholesky', exponent=p)`` = trace(A^-p): p=1 -> ||L^-1||_F^2,
  p=2 -> ||A^-1||_F^2 (A symmetric)
* ``trace(A, exponent=p)`` (method 'exact') = trace(A^p): p=0 -> n
* ``trace(A, method='eigenvalue', eigenvalues=lam, exponent=p)`` = sum(lam^p)

The stochastic ``hutchinson`` / ``slq`` estimators are not restated (parity
unpinned at that boundary; the reference's slq branches are also broken by the
``K_afm`` typo).

This module is also importable under the name ``imate`` by
tests/golden/make_golden.py so that the reference's own MixedCorrelation can run
in the development container.
"""

import numpy
import scipy.linalg
import scipy.sparse


class AffineMatrixFunction(object):
    """Placeholder for imate.AffineMatrixFunction (mixed_correlation.py:44); the
    exact methods never use it."""

    def __init__(self, A, B=None):
        self.A = A
        self.B = B


def _dense(A):
    return A.toarray() if scipy.sparse.issparse(A) else numpy.asarray(A)


def _chol(A):
    return scipy.linalg.cholesky(_dense(A), lower=True, check_finite=False)


def logdet(A, method='cholesky', eigenvalues=None, exponent=1, symmetric=True,
           **kwargs):
    if method == 'eigenvalue':
        lam = numpy.asarray(eigenvalues, dtype=float)
        return exponent * numpy.sum(numpy.log(lam)), {}
    if method in ('cholesky', 'hutchinson'):
        L = _chol(A)
        return exponent * 2.0 * numpy.sum(numpy.log(numpy.diag(L))), {}
    raise ValueError('imate_exact: method %r not restated' % method)


def traceinv(A, method='cholesky', eigenvalues=None, exponent=1, symmetric=True,
             **kwargs):
    if method == 'eigenvalue':
        lam = numpy.asarray(eigenvalues, dtype=float)
        return numpy.sum(lam ** (-float(exponent))), {}
    if method == 'cholesky':
        L = _chol(A)
        n = L.shape[0]
        Linv = scipy.linalg.solve_triangular(L, numpy.eye(n), lower=True,
                                             check_finite=False)
        if exponent == 1:
            return numpy.sum(Linv * Linv), {}
        Ainv = Linv.T @ Linv
        if exponent == 2:
            return numpy.sum(Ainv * Ainv), {}
        return numpy.trace(numpy.linalg.matrix_power(Ainv, exponent)), {}
    raise ValueError('imate_exact: method %r not restated' % method)


def trace(A, method='exact', eigenvalues=None, exponent=1, symmetric=True,
          **kwargs):
    if method == 'eigenvalue':
        lam = numpy.asarray(eigenvalues, dtype=float)
        return numpy.sum(lam ** float(exponent)), {}
    D = _dense(A)
    if exponent == 0:
        return float(D.shape[0]), {}
    if exponent == 1:
        return float(numpy.trace(D)), {}
    if exponent == 2:
        return float(numpy.sum(D * D.T)), {}
    return float(numpy.trace(numpy.linalg.matrix_power(D, exponent))), {}
