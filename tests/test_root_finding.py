"""Host drivers of the profiled optimizer (CPU): the batched bracket search
makes the reference's decisions (_root_finding.py:21-148) with fewer batched
calls, and the whole batched profiled driver reproduces the reference's
recorded optimum and evaluation sequence (tests/golden n1024: bracket found,
Chandrupatla; cfg1: no bracket) with the oracle's exact operator standing in
for the device one."""

import contextlib
import io

import numpy
import pytest

from gaussian_proc._likelihood._root_finding import (
    find_interval_with_sign_change, find_interval_with_sign_change_batched, BatchedFunction,
    chandrupatla_method)
from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood
from oracle.mixed_correlation import MixedCorrelation as OracleMC
from oracle import matern
from _util import check_der1_sequence, load_json, config_inputs

FUNCS = [
    lambda x: x - 0.3,                          # bracket at once
    lambda x: (x - 0.25) * (x - 0.9) + 0.01,    # no sign change in [-4, 3]
    lambda x: numpy.exp(-x) - 0.05,             # root near 3.0
    lambda x: -(x + 3.7) * (x - 2.9),           # both ends negative, roots inside
    lambda x: numpy.tanh(x - 4.2),              # root outside, found by an outward probe
    lambda x: numpy.tanh(-x - 5.5),             # root outside on the left
    lambda x: 1.0 + 0.0 * x,                    # never
    lambda x: (x - 1.0) ** 2 - 1e-3,            # roots close together
]


@pytest.mark.parametrize('k', range(len(FUNCS)))
@pytest.mark.parametrize('bracket', [(-4.0, 3.0), (-1.0, 1.0), (2.0, 5.0)])
def test_batched_bracket_search_makes_the_reference_decisions(k, bracket):
    f = FUNCS[k]
    calls = []

    def fs(x):
        calls.append(x)
        return float(f(x))
    with contextlib.redirect_stdout(io.StringIO()) as out1:
        ref = find_interval_with_sign_change(fs, list(bracket), 3)
    fb = BatchedFunction(lambda xs: numpy.array([f(x) for x in xs]))
    with contextlib.redirect_stdout(io.StringIO()) as out2:
        got = find_interval_with_sign_change_batched(fb, list(bracket), 3)
    assert got == ref
    assert out1.getvalue() == out2.getvalue()          # same diagnostic prints
    assert set(calls) <= set(fb.memo)                  # every point the reference used
    assert fb.calls <= 1 + 3                            # one batch per trial at most
    if ref[0]:
        r1 = chandrupatla_method(fs, ref[1], ref[2], eps_m=1e-6, eps_a=1e-6, maxiter=100)
        r2 = chandrupatla_method(fb, got[1], got[2], eps_m=1e-6, eps_a=1e-6, maxiter=100)
        assert r1 == r2


def _profiled(cfg_name, nu):
    cfg = load_json(cfg_name)
    pts, z, X = config_inputs(cfg)
    K = matern.dense_correlation(pts, cfg['correlation_scale'], nu)
    op = OracleMC(K, 'eigenvalue')
    with contextlib.redirect_stdout(io.StringIO()):
        res = ProfileLikelihood.find_log_likelihood_der1_zeros(z, X, op, [1e-4, 1e3])
    return cfg, res


def test_profiled_driver_bracket_found_matches_reference_n1024():
    cfg, res = _profiled('n1024_nu25.json', 2.5)
    ref = cfg['maximize_profiled']
    assert cfg['maximize_profiled_bracket_found']
    for k in ('sigma', 'sigma0', 'eta'):
        assert abs(res[k] - ref[k]) <= 1e-8 * abs(ref[k]), (k, res[k], ref[k])
    calls, points, memo = ProfileLikelihood.last_der1_calls
    seq = cfg['maximize_profiled_der1_calls']
    scale = max(abs(v) for _, v in seq)
    check_der1_sequence(memo, seq)
    assert calls < len(seq)                 # fewer (batched) calls than reference evals


def test_profiled_driver_no_bracket_matches_reference_cfg1():
    cfg, res = _profiled('cfg1.json', 1.5)
    ref = cfg['maximize_profiled']
    assert res['eta'] == numpy.inf and res['sigma'] == 0
    assert abs(res['sigma0'] - ref['sigma0']) <= 1e-12 * ref['sigma0']


def _raising(f, lo, hi, log):
    """f on [lo, hi]; LinAlgError outside (K + eta I indefinite there)."""
    def fb(xs):
        xs = numpy.asarray(xs, dtype=float)
        log.append(xs.size)
        if numpy.any((xs < lo) | (xs > hi)):
            raise numpy.linalg.LinAlgError('not positive definite')
        return numpy.array([f(x) for x in xs])
    return fb


@pytest.mark.parametrize('k', [0, 2, 3])
def test_speculative_points_outside_the_domain_do_not_fail_the_search(k):
    """The outward probes and Chandrupatla candidates are speculative: a
    function that raises outside [x0, x1] (where the reference never looks
    when the bracket is found inside) gives the reference's result."""
    f = FUNCS[k]
    bracket = (-4.0, 3.0)
    with contextlib.redirect_stdout(io.StringIO()):
        ref = find_interval_with_sign_change(lambda x: float(f(x)), list(bracket), 3)
    assert ref[0]
    log = []
    fb = BatchedFunction(_raising(f, -4.0, 3.0, log), spec_budget=32)
    with contextlib.redirect_stdout(io.StringIO()):
        got = find_interval_with_sign_change_batched(fb, list(bracket), 3, tol=1e-6)
    assert got == ref
    assert fb.spec_failures >= 1                      # the outward probes raised
    r1 = chandrupatla_method(lambda x: float(f(x)), ref[1], ref[2], eps_m=1e-6, eps_a=1e-6,
                             maxiter=100)
    r2 = chandrupatla_method(fb, got[1], got[2], eps_m=1e-6, eps_a=1e-6, maxiter=100)
    assert r1 == r2


@pytest.mark.parametrize('k', [0, 2, 4, 5])
def test_speculative_chandrupatla_same_root_fewer_calls(k):
    """Chandrupatla on a BatchedFunction prefetches the bisection / clamped
    candidates of the next iterations: the same root and iteration count as
    the sequential method, every point it evaluated among the prefetched ones,
    and fewer batched calls than its evaluations."""
    f = FUNCS[k]
    with contextlib.redirect_stdout(io.StringIO()):
        found, br, vals = find_interval_with_sign_change(lambda x: float(f(x)), [-4.0, 3.0], 3)
    assert found
    seq = []

    def fs(x):
        seq.append(x)
        return float(f(x))
    r1 = chandrupatla_method(fs, br, vals, eps_m=1e-6, eps_a=1e-6, maxiter=100)
    fb = BatchedFunction(lambda xs: numpy.array([f(x) for x in xs]), spec_budget=64)
    r2 = chandrupatla_method(fb, br, vals, eps_m=1e-6, eps_a=1e-6, maxiter=100)
    assert r1 == r2
    assert set(seq) <= set(fb.memo)
    assert fb.calls < len(seq), (fb.calls, len(seq))


def test_profiled_driver_speculative_n1024():
    """The profiled driver with speculation on (the band operator's default,
    forced here on the oracle operator): the reference's optimum, its recorded
    evaluation sequence among the evaluated points, at most 2/3 of its
    evaluations as batched calls."""
    cfg = load_json('n1024_nu25.json')
    pts, z, X = config_inputs(cfg)
    K = matern.dense_correlation(pts, cfg['correlation_scale'], 2.5)

    class _Spectral(object):
        """K = U diag(lam) U^T once; solve and traceinv at any eta in O(n^2 m)."""
        imate_method = 'cholesky'     # not the band operator: the duck-type formulas

        def __init__(self, K):
            self.lam, self.U = numpy.linalg.eigh(K)

        def solve(self, eta, Y):
            return self.U @ ((self.U.T @ Y).T / (self.lam + eta)).T

        def traceinv(self, eta, exponent=1):
            return float(numpy.sum((self.lam + eta) ** -exponent))
    op = _Spectral(K)
    with contextlib.redirect_stdout(io.StringIO()):
        res = ProfileLikelihood.find_log_likelihood_der1_zeros(z, X, op, [1e-4, 1e3],
                                                               speculative=24)
    ref = cfg['maximize_profiled']
    for k in ('sigma', 'sigma0', 'eta'):
        assert abs(res[k] - ref[k]) <= 1e-8 * abs(ref[k]), (k, res[k], ref[k])
    calls, points, memo = ProfileLikelihood.last_der1_calls
    seq = cfg['maximize_profiled_der1_calls']
    check_der1_sequence(memo, seq)
    assert 3 * calls <= 2 * len(seq), (calls, len(seq))
    # speculation never makes a call larger than its budget (24 here)
    assert ProfileLikelihood.last_der1_max_batch <= 24


def test_speculative_batches_stay_within_the_budget():
    """Required plus speculative points of every call stay within spec_budget
    (the band operator's 64 is gpmi_band_der_terms' cyclic-reduction limit):
    the bracket search's first call (x0, x1 + 4 probes + Chandrupatla tree)
    and every Chandrupatla step (xt + its candidate tree)."""
    from gaussian_proc._likelihood._root_finding import (BatchedFunction, chandrupatla_method,
                                                         find_interval_with_sign_change_batched)
    sizes = []

    def fbatch(xs):
        sizes.append(len(xs))
        return numpy.tanh(numpy.asarray(xs) - 0.3123)
    for budget in (8, 64):
        sizes.clear()
        fb = BatchedFunction(fbatch, spec_budget=budget)
        found, bracket, values = find_interval_with_sign_change_batched(fb, [-2.0, 3.0], 8,
                                                                        tol=1e-9)
        assert found
        res = chandrupatla_method(fb, bracket, values, eps_m=1e-9, eps_a=1e-9)
        assert abs(res['root'] - 0.3123) < 1e-8
        assert max(sizes) <= budget and fb.max_points == max(sizes), (budget, sizes)
