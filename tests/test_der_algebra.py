"""Host algebra of the band-path eta-derivatives (CPU, no device).

ProfileLikelihood on the dense eigenvalue operator computes der1 / der2 from the
Gram blocks Gp = [X z]^T (K + eta I)^-p [X z] (p = 1..3) and tr((K + eta I)^-1),
tr((K + eta I)^-2) (_profile_likelihood._der_from_terms). Here the blocks come
from numpy and the result is checked against the oracle's restatement of the
reference formulas (_profile_likelihood.py:91-192, oracle/likelihood.py).
"""
import numpy
import pytest

from oracle import matern
from oracle import likelihood as olik
from oracle.mixed_correlation import MixedCorrelation as OracleMC
from _util import rel


def _inputs(n, seed):
    rng = numpy.random.RandomState(seed)
    pts = rng.rand(n, 2)
    K = matern.dense_correlation(pts, 0.2, 1.5)
    X = numpy.column_stack([numpy.ones(n), pts, pts[:, 0] * pts[:, 1]])
    z = numpy.sin(3 * pts[:, 0]) + 0.1 * rng.randn(n)
    return K, X, z


@pytest.mark.parametrize('n,seed', [(60, 1), (250, 2)])
def test_der_from_gram_blocks_matches_reference_formulas(n, seed):
    from gaussian_proc._likelihood._profile_likelihood import _der_from_terms
    K, X, z = _inputs(n, seed)
    m = X.shape[1]
    R = numpy.column_stack([X, z])
    op = OracleMC(K, 'cholesky')
    for eta in (1e-3, 0.07, 1.0, 30.0):
        S = K + eta * numpy.eye(n)
        Si = numpy.linalg.inv(S)
        G1 = R.T @ Si @ R
        G2 = R.T @ Si @ Si @ R
        G3 = R.T @ Si @ Si @ Si @ R
        d1, d2 = _der_from_terms(n, m, G1, G2, G3, numpy.trace(Si), numpy.sum(Si * Si))
        assert rel(d1, olik.profile_der1_eta(z, X, op, numpy.log10(eta))) < 1e-9, eta
        assert rel(d2, olik.profile_der2_eta(z, X, op, eta)) < 1e-8, eta
        d1b, none = _der_from_terms(n, m, G1, G2, G3, numpy.trace(Si))
        assert d1b == d1 and none is None


@pytest.mark.parametrize('n,seed', [(60, 3), (250, 4)])
def test_direct_jac_hess_from_gram_blocks(n, seed):
    """DirectLikelihood Jacobian / Hessian from the Gram blocks vs the oracle's
    restatement of _direct_likelihood.py:89-270."""
    from gaussian_proc._likelihood._direct_likelihood import _jac_hess_from_terms
    K, X, z = _inputs(n, seed)
    m = X.shape[1]
    R = numpy.column_stack([X, z])
    op = OracleMC(K, 'cholesky')
    for sigma, sigma0 in ((0.7, 0.05), (1.3, 0.9), (0.2, 2.5)):
        eta = (sigma0 / sigma) ** 2
        Si = numpy.linalg.inv(K + eta * numpy.eye(n))
        G1, G2, G3 = (R.T @ P @ R for P in (Si, Si @ Si, Si @ Si @ Si))
        jac, hess = _jac_hess_from_terms(n, m, sigma, eta, G1, G2, G3, numpy.trace(Si),
                                         numpy.sum(Si * Si))
        assert rel(jac, olik.direct_jac(z, X, op, [sigma, sigma0])) < 1e-9
        assert rel(hess, olik.direct_hess(z, X, op, [sigma, sigma0])) < 1e-8


def test_direct_band_forms_refuse_cancellation():
    """At eta far above K's spectrum the K-weighted forms Q1 - eta Q2 ... cancel:
    _jac_hess_from_terms returns None and the caller takes the solve path."""
    from gaussian_proc._likelihood._direct_likelihood import _jac_hess_from_terms
    K, X, z = _inputs(60, 5)
    m, n = X.shape[1], 60
    R = numpy.column_stack([X, z])
    eta = 1.6e17
    Si = numpy.linalg.inv(K + eta * numpy.eye(n))
    G1, G2, G3 = (R.T @ P @ R for P in (Si, Si @ Si, Si @ Si @ Si))
    assert _jac_hess_from_terms(n, m, 1e-9, eta, G1, G2, G3, numpy.trace(Si),
                                numpy.sum(Si * Si)) == (None, None)
