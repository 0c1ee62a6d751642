"""traceinv interpolation (MixedCorrelation(interpolate=True); the reference's
imate.InterpolateTraceInv, mixed_correlation.py:52-66,167-170). imate is absent:
parity unpinned. Checked here on the CPU against exact traceinv from numpy
eigenvalues: exact at the interpolant points, the exact large-eta limit, and a
bounded error between the points."""

import numpy

from gaussian_proc._mixed_correlation._interpolate import InterpolateTraceInv
from oracle import matern


def _exact(seed=3, n=400, nu=1.5, scale=0.15):
    rng = numpy.random.RandomState(seed)
    K = matern.dense_correlation(rng.rand(n, 2), scale, nu)
    lam = numpy.linalg.eigvalsh(K)
    return K, lam, (lambda t: float(numpy.sum(1.0 / (lam + t))))


def test_interpolant_is_exact_at_points_and_at_infinity():
    K, lam, tr = _exact()
    pts = [1e-3, 1e-2, 1e-1, 1.0, 10.0]
    it = InterpolateTraceInv(tr, K.shape[0], numpy.trace(K), pts)
    for t in pts:
        assert abs(it.interpolate(t) - tr(t)) <= 1e-12 * tr(t)
    for t, tol in ((1e4, 1e-4), (1e7, 1e-10)):
        assert abs(it.interpolate(t) - tr(t)) <= tol * tr(t)


def test_interpolant_between_points():
    K, lam, tr = _exact()
    pts = numpy.logspace(-3, 2, 11)
    it = InterpolateTraceInv(tr, K.shape[0], numpy.trace(K), pts)
    grid = numpy.logspace(-3, 2, 200)
    err = max(abs(it.interpolate(t) - tr(t)) / tr(t) for t in grid)
    assert err < 2e-2, err
    # a denser set of points converges
    it2 = InterpolateTraceInv(tr, K.shape[0], numpy.trace(K), numpy.logspace(-3, 2, 41))
    err2 = max(abs(it2.interpolate(t) - tr(t)) / tr(t) for t in grid)
    assert err2 < err / 4, (err2, err)


def test_interpolant_uses_the_callers_points():
    """The chosen semantics ("Interpolation"): the interpolant's
    nodes are the caller's interpolant_points (the reference requires them but
    never forwards them to imate, which then uses its own defaults): its nodes are
    exactly those points, it is exact at each, and a different point set gives a
    different interpolant between them."""
    K, lam, tr = _exact()
    pts_a = [1e-2, 1.0, 100.0]
    pts_b = [1e-3, 1e-1, 10.0]
    ia = InterpolateTraceInv(tr, K.shape[0], numpy.trace(K), pts_a)
    ib = InterpolateTraceInv(tr, K.shape[0], numpy.trace(K), pts_b)
    numpy.testing.assert_array_equal(ia.points, pts_a)
    numpy.testing.assert_array_equal(ib.points, pts_b)
    for t in pts_a:
        assert abs(ia.interpolate(t) - tr(t)) <= 1e-12 * tr(t)
    for t in pts_b:
        assert abs(ib.interpolate(t) - tr(t)) <= 1e-12 * tr(t)
    assert abs(ia.interpolate(0.1) - ib.interpolate(0.1)) > 1e-9 * tr(0.1)
