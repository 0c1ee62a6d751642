"""imate 'slq' on a DENSE K (mixed_correlation.py:138-143,204-209,263-268):
the device Krylov primitives over the resident dense matrix
(gpmi_sp_create_dense, dense_mm_kernel on fp64 MFMA).

The reference's own dense 'slq' branch passes the misspelt ``self.K_afm`` and
raises AttributeError, so no reference value exists (parity unpinned). The
checks are therefore against the oracle and exact values:
- K X (+ eta X) vs numpy, ragged n, s = 1 .. 40 columns: <= 1e-13 relative
  (summation order differs from numpy's; fp64 throughout);
- the device Lanczos vs the oracle's CGS2 Lanczos with the same counter-based
  probes: alpha / beta and the SLQ sums <= 1e-9 relative (as on a sparse K);
- SLQ logdet / traceinv vs the exact values (dense Cholesky) within 4 standard
  errors of the probe mean; trace exponents 3 and traceinv exponent 3 against
  the eigenvalue sums likewise;
- CG and the multi-shift Gram vs numpy solves (rtol 1e-10 -> <= 1e-8).
"""

import numpy
import pytest

from oracle import data, matern, sparse as osp
from _util import rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def gp():
    import gaussian_proc
    from gaussian_proc import _hip
    _hip.require_device(0)
    return gaussian_proc


def _dense_K(n_side, scale=0.1, nu=1.5):
    pts = data.generate_points(n_side, 2, True)
    return matern.dense_correlation(pts, scale, nu)


def _nrel(a, b):
    return float(numpy.max(numpy.abs(a - b)) / numpy.max(numpy.abs(b)))


@pytest.mark.parametrize('n', [300, 1000, 4133])
def test_dense_mm_matches_numpy(gp, n):
    from gaussian_proc import _hip
    rng = numpy.random.RandomState(n)
    A = rng.randn(n, n)
    K = 0.5 * (A + A.T)
    op = _hip.Operator(n)
    op.load_matrix(K)
    sop = _hip.SparseOperator.from_dense(op)
    assert sop.n == n and sop.nnz == n * n
    assert sop.spmm_kernel(20) == 'dense_mm_kernel'
    for s in (1, 5, 16, 17, 20, 32, 40):
        X = rng.randn(n, s)
        Y = sop.spmm(0.7, X)
        assert _nrel(Y, K @ X + 0.7 * X) < 1e-13, s
    with pytest.raises(_hip.GPMIError):
        sop.csr()


def test_dense_lanczos_matches_oracle_same_probes(gp):
    from gaussian_proc import _hip, _slq
    K = _dense_K(24)
    n = K.shape[0]
    op = _hip.Operator(n)
    op.load_matrix(K)
    sop = _hip.SparseOperator.from_dense(op)
    nprobe, steps, seed = 6, 25, 11
    a, b = sop.lanczos(nprobe, steps, seed)
    P = osp.rademacher_probes(n, nprobe, seed)
    for p in range(nprobe):
        ao, bo = osp.lanczos(K, P[:, p], steps)
        k = ao.size
        assert rel(a[p, :k], ao) < 1e-9
        assert rel(b[p, :k - 1], bo) < 1e-9
    etas = [0.05, 1.0]
    ref = osp.slq(K, etas, P, steps)
    nodes = _slq.nodes(a, b)
    for what in ('logdet', 'traceinv', 'traceinv2'):
        est = n * _slq.quadrature(nodes, etas, _slq.FUNCS[what]).mean(axis=0)
        assert rel(est, ref[what]) < 1e-9, what


@pytest.mark.parametrize('orth', [0, -1])
def test_dense_slq_operator_vs_exact(gp, orth):
    """MixedCorrelation(K, imate_method='slq') on a dense K with imate's
    lanczos_tol: every SLQ quantity within 4 standard errors of its exact value,
    two-sided, down to eta = 0.01 (the Lanczos degree grows from 40 until the
    Gauss / Gauss-Radau gap at the eta asked is within the tolerance; at a fixed
    30 steps traceinv at eta = 0.01 was 14 standard errors low on this smooth
    kernel, at 40 steps 3.8; the tolerance takes it to ~110 steps). imate's default
    plain three-term recurrence (orthogonalize=0) and full reorthogonalisation (-1)."""
    from gaussian_proc import _slq
    from gaussian_proc._mixed_correlation import MixedCorrelation
    K = _dense_K(32)
    n = K.shape[0]
    ns = 64
    op = MixedCorrelation(K, imate_method='slq',
                          imate_options={'num_samples': ns, 'lanczos_degree': 40,
                                         'lanczos_tol': 1e-6, 'orthogonalize': orth})
    lam = numpy.linalg.eigvalsh(K)
    cases = (('logdet', numpy.log, lambda e: op.logdet(e), (0.01, 0.3, 5.0)),
             ('traceinv', lambda x: 1.0 / x, lambda e: op.traceinv(e), (0.01, 0.3, 5.0)),
             ('traceinv3', lambda x: x ** -3.0, lambda e: op.traceinv(e, 3), (0.3, 5.0)),
             ('trace3', lambda x: x ** 3.0, lambda e: op.trace(e, 3), (0.01, 0.3, 5.0)))
    for what, fn, call, etas in cases:
        for eta in etas:
            exact = float(numpy.sum(fn(lam + eta)))
            val = call(eta)
            conv = op.last_slq_convergence
            assert conv['converged'] and conv['bracket'] <= 1e-6, (what, eta, conv)
            per = n * _slq.quadrature(op.slq_nodes(), [eta], fn)[:, 0]
            se = per.std(ddof=1) / numpy.sqrt(ns)
            assert val == pytest.approx(per.mean(), rel=1e-12)
            assert abs(val - exact) <= 4.0 * se + 1e-9 * abs(exact), (what, eta, val, exact, se)
    # the degree grew for the small shift and never shrinks
    assert 40 < op.lanczos_degree_used <= 256
    # exact parts: trace exponents 0-2, dot, solve (dense Cholesky)
    I = numpy.eye(n)
    assert rel(op.trace(0.5, 2), numpy.trace((K + 0.5 * I) @ (K + 0.5 * I))) < 1e-12
    assert op.traceinv(0.5, 0) == n
    x = numpy.arange(n, dtype=float)
    numpy.testing.assert_allclose(op.dot(0.5, x, 2), 2 * (K @ x + 0.5 * x), rtol=1e-12)
    y = op.solve(0.5, x)
    assert _nrel(y, numpy.linalg.solve(K + 0.5 * I, x)) < 1e-10


def test_dense_cg_and_msgram(gp):
    from gaussian_proc import _hip
    K = _dense_K(28)
    n = K.shape[0]
    op = _hip.Operator(n)
    op.load_matrix(K)
    sop = _hip.SparseOperator.from_dense(op)
    rng = numpy.random.RandomState(3)
    B = rng.randn(n, 7)
    eta = 0.5
    Y = sop.cg(eta, B, rtol=1e-12)
    assert _nrel(Y, numpy.linalg.solve(K + eta * numpy.eye(n), B)) < 1e-8
    etas = numpy.array([0.5, 2.0, 30.0])
    G = sop.msgram(etas, B, rtol=1e-10)
    for e, g in zip(etas, G):
        ex = B.T @ numpy.linalg.solve(K + e * numpy.eye(n), B)
        assert _nrel(g, ex) < 1e-8, e


def test_dense_slq_likelihood_sweep(gp):
    """The sparse sweep drivers run unchanged on the dense 'slq' operator:
    sweep.slq_sweep curves equal the operator's own per-eta values, and the
    direct likelihood through SLQ logdet + Cholesky solves is within the SLQ
    error of the exact ('cholesky') likelihood."""
    from gaussian_proc import sweep
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    pts = data.generate_points(32, 2, True)
    K = matern.dense_correlation(pts, 0.1, 1.5)
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    op = MixedCorrelation(K, imate_method='slq',
                          imate_options={'num_samples': 48, 'lanczos_degree': 30})
    etas = numpy.array([0.05, 0.5, 5.0])
    curves = sweep.slq_sweep(op, etas)
    for i, eta in enumerate(etas):
        assert curves['logdet'][i] == pytest.approx(op.logdet(eta), rel=1e-12)
    ex = MixedCorrelation(K, imate_method='cholesky')
    for eta in etas:
        ld_slq, ld_ex = op.logdet(eta), ex.logdet(eta)
        assert abs(ld_slq - ld_ex) < 0.02 * abs(ld_ex) + 2.0
    hyper = [0.5, 0.3]   # sigma, sigma0 -> eta = 0.36
    lp_slq = DirectLikelihood.log_likelihood(z, X, op, False, hyper)
    lp_ex = DirectLikelihood.log_likelihood(z, X, ex, False, hyper)
    # the same Gram blocks (exact solves); only the logdet is estimated
    ld_slq, ld_ex = op.logdet(0.36), ex.logdet(0.36)
    assert lp_slq - lp_ex == pytest.approx(-0.5 * (ld_slq - ld_ex), rel=1e-6, abs=1e-8)
