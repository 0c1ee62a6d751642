"""Host side of the stochastic estimators (CPU): the Gauss-Radau rules of
_slq bracket the exact quadratic form, so their gap bounds the Lanczos part of
the SLQ error (imate's lanczos_tol control), and imate_options are checked
against the keywords imate's functions accept (TypeError otherwise)."""

import numpy
import pytest

from gaussian_proc import _slq


def _lanczos_with_last_beta(K, v, m):
    """Lanczos (CGS2) returning alpha[m] and beta[m], beta[m - 1] the coupling
    to the next vector (the device's convention)."""
    n = K.shape[0]
    V = numpy.zeros((m + 1, n))
    V[0] = v / numpy.linalg.norm(v)
    a, b = [], []
    bp, vp = 0.0, numpy.zeros(n)
    for k in range(m):
        w = K @ V[k] - bp * vp
        for _ in range(2):
            h = V[:k + 1] @ w
            w -= V[:k + 1].T @ h
        a.append(V[k] @ K @ V[k])
        bb = numpy.linalg.norm(w)
        b.append(bb)
        vp, bp = V[k], bb
        V[k + 1] = w / bb
    return numpy.array(a), numpy.array(b)


@pytest.mark.parametrize('m', [5, 12, 25])
def test_gauss_and_radau_bracket_the_quadratic_form(m):
    rng = numpy.random.RandomState(m)
    lam = numpy.sort(rng.gamma(0.3, 2.0, 400)) + 1e-4      # clustered near 0, like a smooth K
    K = numpy.diag(lam)
    P = _slq.rademacher(lam.size, 6, 2)
    ab = [_lanczos_with_last_beta(K, P[:, p], m) for p in range(6)]
    A = numpy.array([a for a, _ in ab])
    B = numpy.array([b for _, b in ab])
    g = _slq.nodes(A, B)
    r = _slq.radau_nodes(A, B, 0.0)
    for fn in (numpy.log, lambda x: 1.0 / x, lambda x: x ** -2.0):
        for eta in (1e-3, 0.1, 2.0):
            exact = numpy.mean([numpy.sum(P[:, p] ** 2 * fn(lam + eta)) / lam.size
                                for p in range(6)])
            G = _slq.quadrature(g, [eta], fn).mean()
            R = _slq.quadrature(r, [eta], fn).mean()
            lo, hi = min(G, R), max(G, R)
            assert lo - 1e-12 * abs(exact) <= exact <= hi + 1e-12 * abs(exact)
            assert abs(G - exact) <= _slq.bracket(g, r, [eta], fn)[0] * abs(G) * (1 + 1e-9) + \
                1e-14 * abs(exact)


def test_radau_of_a_broken_down_probe_is_its_gauss_rule():
    a = numpy.array([[2.0, 1.0, 3.0]])
    b = numpy.array([[0.5, 0.0, 0.0]])      # invariant after two steps: exact rule
    g = _slq.nodes(a, b)
    r = _slq.radau_nodes(a, b, 0.0)
    numpy.testing.assert_array_equal(g[0][0], r[0][0])
    assert _slq.bracket(g, r, [0.1], numpy.log)[0] == 0.0


def test_radau_node_above_the_ritz_values_moves_below_them():
    """A node that is not below a probe's Ritz values (rounding puts a node a hair
    below the smallest one on the wrong side: the last pivot d_m <= 0) is moved
    to that probe's smallest Ritz value minus 1e-8 max|T|: radau_nodes never
    raises (a rank raising alone inside slq_sweep's all-gather would
    leave the other ranks blocked), and the rule still brackets."""
    a = numpy.array([[2.0, 2.0]])
    b = numpy.array([[1.0, 0.5]])
    g = _slq.nodes(a, b)
    for lower in (5.0, float(g[0][0].min()), float(g[0][0].min()) * (1 - 1e-17)):
        r = _slq.radau_nodes(a, b, lower)
        assert r[0][0].size == 3
        assert r[0][0].min() < g[0][0].min()
        assert numpy.all(numpy.isfinite(r[0][1]))


def test_radau_without_a_valid_node_never_reads_converged(monkeypatch):
    """when no Radau node gives a positive last pivot, the probe gets a
    NaN rule (not its Gauss rule, whose zero gap could close the bracket falsely):
    the bracket is inf, so the lanczos_tol searches keep going or report
    unconverged."""
    rng = numpy.random.RandomState(3)
    lam = numpy.sort(rng.gamma(0.3, 2.0, 200)) + 1e-3
    K = numpy.diag(lam)
    P = _slq.rademacher(lam.size, 3, 5)
    ab = [_lanczos_with_last_beta(K, P[:, p], 10) for p in range(3)]
    A = numpy.array([a for a, _ in ab])
    B = numpy.array([b for _, b in ab])
    g = _slq.nodes(A, B)
    monkeypatch.setattr(_slq, '_last_pivot', lambda a, b, lower: -1.0)
    r = _slq.radau_nodes(A, B, 0.0)
    assert all(numpy.isnan(t).all() for t, _ in r)
    gap = _slq.bracket(g, r, [0.1], numpy.log)[0]
    assert gap == numpy.inf and not gap <= 1e-3
    assert _slq.gap(1.0, numpy.nan) == numpy.inf and _slq.gap(2.0, 1.0) == 0.5


def test_nodes_do_not_depend_on_the_probe_grouping():
    """a probe's Ritz nodes are the same whether it is solved alone (a
    rank's shard of one probe) or with others (the whole set at N = 1)."""
    rng = numpy.random.RandomState(7)
    lam = numpy.sort(rng.gamma(0.3, 2.0, 300)) + 1e-3
    K = numpy.diag(lam)
    P = _slq.rademacher(lam.size, 4, 1)
    ab = [_lanczos_with_last_beta(K, P[:, p], 16) for p in range(4)]
    A = numpy.array([a for a, _ in ab])
    B = numpy.array([b for _, b in ab])
    together = _slq.nodes(A, B)
    for p in range(4):
        alone = _slq.nodes(A[p:p + 1], B[p:p + 1])[0]
        numpy.testing.assert_array_equal(alone[0], together[p][0])
        numpy.testing.assert_array_equal(alone[1], together[p][1])


def test_stemr_failure_falls_back_to_dense_eigh():
    """The tridiagonal on which LAPACK stemr stops with info = 22 (a plain Lanczos
    at 130 steps: duplicated Ritz values; tests/golden/make_stemr_fixture.py):
    _slq._rule returns numpy.linalg.eigh's nodes and squared first components."""
    import os
    import scipy.linalg
    z = numpy.load(os.path.join(os.path.dirname(__file__), 'golden', 'stemr_info22.npz'))
    d, e = z['d'], z['e']
    with pytest.raises(numpy.linalg.LinAlgError):
        scipy.linalg.eigh_tridiagonal(d, e)      # the failure the fallback exists for
    theta, w = _slq._rule(d, e)
    T = numpy.diag(d) + numpy.diag(e, 1) + numpy.diag(e, -1)
    lam, U = numpy.linalg.eigh(T)
    numpy.testing.assert_array_equal(theta, lam)
    numpy.testing.assert_array_equal(w, U[0] ** 2)
    assert abs(w.sum() - 1.0) < 1e-12
    # nodes() goes through the same rule (one probe, beta padded to the steps)
    nd = _slq.nodes(d[None, :], numpy.append(e, 1.0)[None, :])
    numpy.testing.assert_array_equal(nd[0][0], lam)


def test_radau_node_choice_keeps_f_finite():
    """a sparse tapered K's Gershgorin bound lies far below -min(eta),
    where log / inverse powers are NaN or infinite. radau_node then takes the
    smallest Ritz value minus a margin (flagged not rigorous); a bound with
    lower + min(eta) > 0 is kept (rigorous)."""
    nodes = [(numpy.array([-0.2, 0.5, 3.0]), numpy.array([0.2, 0.3, 0.5]))]
    node, rig = _slq.radau_node(-5.0, nodes, [0.3, 1.0])
    assert not rig and -0.3 < node < -0.2
    assert numpy.isfinite(numpy.log(node + 0.3))
    node, rig = _slq.radau_node(-0.25, nodes, [0.3])
    assert rig and node == -0.25
    # the margin would cross -min(eta): half-way between
    node, rig = _slq.radau_node(-5.0, nodes, [0.2 + 1e-12])
    assert not rig and -0.2 - 1e-12 < node < -0.2


@pytest.mark.parametrize('method,options', [
    ('slq', {'lanczos_degree': 10, 'bogus': 1}),
    ('slq', {'exponent': 2}),                 # the reference passes it itself
    ('hutchinson', {'lanczos_degree': 20}),
    ('cholesky', {'num_samples': 5}),
    ('eigenvalue', {'eigenvalues': None}),
])
def test_unknown_imate_options_raise_type_error(method, options):
    """imate's keyword functions take no other keys than their own: a key that
    no imate function of the method accepts is a TypeError at construction
    (before any device work)."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    with pytest.raises(TypeError, match='unexpected keyword'):
        MixedCorrelation(numpy.eye(4), imate_method=method, imate_options=options)


def test_known_imate_options_pass_the_check():
    from gaussian_proc._mixed_correlation.mixed_correlation import _check_options
    _check_options('slq', {'min_num_samples': 5, 'max_num_samples': 9, 'error_rtol': 1e-2,
                           'lanczos_degree': 20, 'lanczos_tol': 1e-6, 'orthogonalize': 0,
                           'num_samples': 8, 'max_lanczos_degree': 64})
    _check_options('hutchinson', {'solver_tol': 1e-8, 'orthogonalize': False, 'seed': 3})
    _check_options('cholesky', {'cholmod': None, 'invert_cholesky': True})
    _check_options('eigenvalue', {'non_zero_ratio': 0.9, 'tol': 1e-3})


def test_next_lanczos_degree_extrapolates_the_gap():
    """The lanczos_tol search: the first retry doubles the degree; with two gaps
    the next degree is where the line through their logarithms reaches the
    tolerance (+10 %, a multiple of 8), never fewer than 8 more steps."""
    from gaussian_proc._mixed_correlation.mixed_correlation import _next_degree
    assert _next_degree([(30, 0.46)], 1e-3) == 60
    m = _next_degree([(30, 0.46), (60, 0.195)], 1e-3)
    rate = numpy.log(0.46 / 0.195) / 30.0
    want = 60 + numpy.log(0.195 / 1e-3) / rate
    assert m % 8 == 0 and 1.1 * want <= m < 1.1 * want + 8
    assert _next_degree([(40, 1e-3), (48, 2e-3)], 1e-6) == 96      # gap grew: double
    assert _next_degree([(40, 1e-5), (80, 1.01e-6)], 1e-6) == 96   # 1.1 x 80.2, rounded up
    assert _next_degree([(40, 1e-5), (41, 1e-12)], 1e-6) == 49     # at least 8 more


def test_quadrature_batched_equals_per_probe_bits():
    """_slq.quadrature forms every probe's sums in one array op when the rules have
    one length (round 6); the values are the per-probe loop's bits. Ragged rules
    (a probe that broke down early) take the per-probe loop."""
    from gaussian_proc import _slq
    rng = numpy.random.RandomState(4)
    etas = numpy.logspace(-2, 2, 32)
    for k in (1, 7, 30, 61):
        nodes = [(numpy.sort(rng.rand(k) * 3 + 0.1), rng.rand(k)) for _ in range(20)]
        for fn in _slq.FUNCS.values():
            ref = numpy.array([numpy.sum(w[None, :] * fn(t[None, :] + etas[:, None]), axis=1)
                               for t, w in nodes])
            numpy.testing.assert_array_equal(_slq.quadrature(nodes, etas, fn, check=False), ref)
    ragged = [(numpy.sort(rng.rand(k) * 3 + 0.1), rng.rand(k)) for k in (30, 12, 30)]
    q = _slq.quadrature(ragged, etas, numpy.log, check=False)
    for p, (t, w) in enumerate(ragged):
        numpy.testing.assert_array_equal(
            q[p], numpy.sum(w[None, :] * numpy.log(t[None, :] + etas[:, None]), axis=1))
