"""Band path (imate_method='eigenvalue' operator) on an MI355X vs the oracle.

The device reduces K once to band form K = Q B Q^T (bandwidth 128), then every
eta is a banded Cholesky of B + eta I (csrc/gpmi_band.hip). Checks: B is
orthogonally similar to K (same spectrum), logdet and R^T (K + eta I)^-1 R vs
the CPU restatement at ragged sizes (logdet <= 1e-10 rel), the cfg2 / cfg3
golden vectors of the reference's eigenvalue operator (logdet <= 1e-9 rel, lp <=
1e-8 rel), many eta in one call, and the not-SPD error.
"""

import numpy
import pytest

from oracle import matern
from oracle.mixed_correlation import MixedCorrelation as OracleMC
from _util import load_json, config_inputs, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def gp():
    import gaussian_proc
    from gaussian_proc import _hip
    _hip.require_device(0)
    return gaussian_proc


def _mc(K, **kw):
    from gaussian_proc._mixed_correlation import MixedCorrelation
    return MixedCorrelation(K, imate_method='eigenvalue', **kw)


def _inputs(n, seed, nu=1.5, scale=0.2):
    rng = numpy.random.RandomState(seed)
    pts = rng.rand(n, 2)
    K = matern.dense_correlation(pts, scale, nu)
    X = numpy.column_stack([numpy.ones(n), pts])
    z = numpy.sin(3 * pts[:, 0]) + 0.1 * rng.randn(n)
    return K, X, z


@pytest.mark.parametrize('n', [129, 300, 1000])
def test_band_is_orthogonally_similar(gp, n):
    K, _, _ = _inputs(n, n)
    op = _mc(K)
    B = op.band().band()
    i, j = numpy.indices(B.shape)
    assert numpy.all(B[numpy.abs(i - j) > 128] == 0.0)
    numpy.testing.assert_array_equal(B, B.T)
    lam_K = numpy.linalg.eigvalsh(K)
    lam_B = numpy.linalg.eigvalsh(B)
    assert numpy.max(numpy.abs(lam_B - lam_K)) <= 1e-12 * numpy.abs(lam_K).max()


@pytest.mark.parametrize('n', [1, 5, 127, 128, 129, 300, 1000])
def test_band_loglik_terms_vs_oracle(gp, n):
    K, X, z = _inputs(n, n + 1)
    op = _mc(K)
    ref = OracleMC(K, 'cholesky')
    etas = [1e-2, 0.05, 0.5, 5.0]
    ld, G = op.loglik_terms(etas, X, z)
    R = numpy.column_stack([X, z])
    for e, l, g in zip(etas, ld, G):
        assert rel(l, ref.logdet(e)) < 1e-10, (n, e)
        numpy.testing.assert_allclose(g, R.T @ ref.solve(e, R), rtol=1e-8, atol=1e-10)
    assert rel(op.logdet(0.3), ref.logdet(0.3)) < 1e-10


def test_band_many_etas_one_call(gp):
    K, X, z = _inputs(600, 11, nu=2.5, scale=0.1)
    op = _mc(K)
    etas = numpy.logspace(-3, 3, 300)
    ld, G = op.loglik_terms(etas, X, z)
    chol = _mc(K)
    chol.imate_method = 'cholesky'
    ld_c, G_c = chol.loglik_terms(etas[::37], X, z)
    assert rel(ld[::37], ld_c) < 1e-10
    numpy.testing.assert_allclose(G[::37], G_c, rtol=1e-8, atol=1e-10)


def test_band_cfg2_golden(gp):
    """N=4096 (config 2) vs the reference's eigenvalue operator and direct lp."""
    cfg = load_json('cfg2.json')
    pts, z, X = config_inputs(cfg)
    D = gp.generate_correlation(pts, 0.1, 1.5, device_resident=True)
    op = _mc(D)
    assert rel([op.logdet(e) for e in cfg['etas']], cfg['operator']['eigenvalue']['logdet']) < 1e-9
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    lp = DirectLikelihood.log_likelihood_batch(z, X, op, cfg['hypers'])
    assert rel(lp, cfg['direct_lp']) < 1e-8
    t = op.band().last_timing()
    assert t['reduce_ms'] > 0 and t['loglik_ms'] > 0


def test_band_not_positive_definite(gp):
    n = 300
    rng = numpy.random.RandomState(3)
    A = rng.randn(n, n)
    op = _mc(A + A.T)
    with pytest.raises(numpy.linalg.LinAlgError):
        op.logdet(0.0)
    ref = OracleMC(A + A.T)
    assert rel(op.logdet(100.0), ref.logdet(100.0)) < 1e-10


@pytest.mark.slow
def test_band_cfg3_n16384(gp):
    """N=16384 (config 3, metric variant nu=1.5): logdet and direct lp of the
    64-point grid's golden subset from one band reduction."""
    cfg = load_json('cfg3_big.json')
    from oracle import data
    pts = data.generate_points(128, 2, True)
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    D = gp.generate_correlation(pts, 0.1, 1.5, device_resident=True)
    op = _mc(D)
    ld, _ = op.loglik_terms(cfg['etas'], X, z)
    assert rel(ld, cfg['logdet']) < 1e-9
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    lp = DirectLikelihood.log_likelihood_batch(z, X, op, cfg['hypers'])
    assert rel(lp, cfg['direct_lp']) < 1e-8


def test_dense_hutchinson_traceinv_within_mc_error(gp):
    """'hutchinson' traceinv on a dense K (Rademacher probes, device Cholesky
    solves): stochastic, so checked against the exact trace within 4 standard
    errors of the estimator (imate is absent: parity unpinned)."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    K, _, _ = _inputs(400, 9)
    s = 200
    op = MixedCorrelation(K, imate_method='hutchinson', imate_options={'num_samples': s})
    for eta in (0.1, 1.0):
        Ainv = numpy.linalg.inv(K + eta * numpy.eye(400))
        exact = numpy.trace(Ainv)
        # Var of the Rademacher estimator: 2 (||A^-1||_F^2 - sum diag^2) / s
        se = numpy.sqrt(2.0 * (numpy.sum(Ainv ** 2) - numpy.sum(numpy.diag(Ainv) ** 2)) / s)
        assert abs(op.traceinv(eta) - exact) < 4 * se + 1e-12
        assert op.logdet(eta) == pytest.approx(numpy.linalg.slogdet(K + eta * numpy.eye(400))[1],
                                               rel=1e-10)


@pytest.mark.parametrize('orth', [True, False])
def test_dense_hutchinson_traceinv_exponent_3_and_4(gp, orth):
    """'hutchinson' traceinv of exponent 3 (two chained device solves per probe:
    u = A^-1 v, u^T A^-1 u) and 4 (|A^-2 v|^2) within 4 standard errors of the
    eigenvalue sum; imate's orthogonalize option on and off."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    K, _, _ = _inputs(400, 9)
    s = 200
    op = MixedCorrelation(K, imate_method='hutchinson',
                          imate_options={'num_samples': s, 'orthogonalize': orth})
    lam = numpy.linalg.eigvalsh(K)
    for p in (3, 4):
        for eta in (0.5, 2.0):
            B = numpy.linalg.matrix_power(numpy.linalg.inv(K + eta * numpy.eye(400)), p)
            se = numpy.sqrt(2.0 * (numpy.sum(B ** 2) - numpy.sum(numpy.diag(B) ** 2)) / s)
            exact = numpy.sum((lam + eta) ** -float(p))
            assert abs(op.traceinv(eta, p) - exact) < 4 * se + 1e-12 * exact, (p, eta)
    assert op.traceinv(1.0, 0) == 400
    with pytest.raises(ValueError):
        op.traceinv(1.0, 1.5)


@pytest.mark.parametrize('n', [2, 5, 129, 300, 1000])
def test_eigenvalues_vs_numpy(gp, n):
    """Device bulge chase + bisection: the spectrum of K to 1e-12 ||K||."""
    K, _, _ = _inputs(n, n + 2)
    lam = _mc(K).eigenvalues()
    ref = numpy.linalg.eigvalsh(K)
    assert lam.shape == (n,)
    assert numpy.all(numpy.diff(lam) >= 0)
    assert numpy.max(numpy.abs(lam - ref)) <= 1e-12 * numpy.abs(ref).max()


@pytest.mark.parametrize('n', [3, 130, 1000, 2177])
def test_systolic_chase_matches_launch_form(gp, n, monkeypatch):
    """The one-launch systolic chase (default: a D and an E workgroup per chase
    position; also one workgroup per position) and the per-wavefront launch form
    give the same tridiagonal up to rounding (sums in another order): the
    spectra agree to 1e-13 ||K|| and match numpy to 1e-12 ||K||."""
    K, _, _ = _inputs(n, n + 3)
    op = _mc(K)
    lam = op.eigenvalues()
    info = op.band().chase_info()
    assert info['systolic'] == 2 and info['fallbacks'] == 0, info   # D / E workgroups
    monkeypatch.setenv('GPMI_CHASE_MODE', 'systolic')                # one per position
    b1 = _mc(K).band()
    lam_1 = b1.eigenvalues()
    assert b1.chase_info()['systolic'] == 1
    monkeypatch.setenv('GPMI_CHASE_MODE', 'split')                   # launch form
    lam_s = _mc(K).band().eigenvalues()
    ref = numpy.linalg.eigvalsh(K)
    scale = numpy.abs(ref).max()
    assert numpy.max(numpy.abs(lam - lam_s)) <= 1e-13 * scale
    assert numpy.max(numpy.abs(lam_1 - lam_s)) <= 1e-13 * scale
    assert numpy.max(numpy.abs(lam - ref)) <= 1e-12 * scale


def test_multisection_matches_bisection(gp, monkeypatch):
    """Multisection (16 Sturm counts per round, default) and one-thread bisection
    find every eigenvalue to the same 2-ulp interval: they agree to 4 ulp of
    max |lambda|."""
    K, _, _ = _inputs(1500, 8)
    lam = _mc(K).eigenvalues()
    monkeypatch.setenv('GPMI_BISECT', '1')
    lam_b = _mc(K).eigenvalues()
    scale = numpy.abs(lam_b).max()
    assert numpy.max(numpy.abs(lam - lam_b)) <= 8.9e-16 * scale


def test_chase_over_split_capacity_uses_one_workgroup_per_position(gp, monkeypatch):
    """N = 129^2 = 16641 needs 2 x 130 split-chase workgroups, more than 256 CUs
    hold: the one-workgroup-per-position systolic kernel takes over (no timeout)
    and agrees with the launch form to 1e-13 max |lambda|."""
    from oracle import data
    pts = data.generate_points(129, 2, True)
    D = gp.generate_correlation(pts, 0.1, 1.5, device_resident=True)
    b = _mc(D).band()
    lam = b.eigenvalues()
    info = b.chase_info()
    if 2 * 130 <= info['maxg']:
        pytest.skip('this device holds the split chase at N = 16641')
    assert info['systolic'] == 1 and info['fallbacks'] == 0, info
    monkeypatch.setenv('GPMI_CHASE_MODE', 'split')
    lam_s = _mc(D).band().eigenvalues()
    assert numpy.max(numpy.abs(lam - lam_s)) <= 1e-13 * numpy.abs(lam_s).max()


def test_systolic_chase_timeout_falls_back(gp, monkeypatch):
    """GPMI_CHASE_SPIN_LIMIT=0 makes the first hand-off wait of the systolic
    chase a timeout (as when its workgroups cannot all be resident): every
    workgroup leaves, the launch form reruns the chase, the spectrum is right
    and the fallback is counted."""
    K, _, _ = _inputs(1000, 5)
    monkeypatch.setenv('GPMI_CHASE_SPIN_LIMIT', '0')
    op = _mc(K)
    lam = op.eigenvalues()
    info = op.band().chase_info()
    assert info['systolic'] == 0 and info['fallbacks'] == 2, info   # split, then one per position
    ref = numpy.linalg.eigvalsh(K)
    assert numpy.max(numpy.abs(lam - ref)) <= 1e-12 * numpy.abs(ref).max()


def test_eigenvalue_operator_traces(gp):
    """'eigenvalue' traceinv (exponent 1, 2, 3) and trace (exponent 3) as sums over
    the device eigenvalues vs explicit matrix functions (rel <= 1e-9)."""
    K, _, _ = _inputs(500, 21, nu=2.5, scale=0.1)
    op = _mc(K)
    for eta in (1e-2, 0.3, 4.0):
        A = K + eta * numpy.eye(500)
        Ainv = numpy.linalg.inv(A)
        assert rel(op.traceinv(eta), numpy.trace(Ainv)) < 1e-9
        assert rel(op.traceinv(eta, 2), numpy.sum(Ainv * Ainv)) < 1e-9
        assert rel(op.traceinv(eta, 3), numpy.trace(Ainv @ Ainv @ Ainv)) < 1e-9
        assert rel(op.trace(eta, 3), numpy.trace(A @ A @ A)) < 1e-9
        assert op.traceinv(eta, 0) == 500


def test_eigenvalue_operator_cfg2_golden(gp):
    """N=4096: traceinv of the reference's eigenvalue operator (golden)."""
    cfg = load_json('cfg2.json')
    pts, z, X = config_inputs(cfg)
    D = gp.generate_correlation(pts, 0.1, 1.5, device_resident=True)
    op = _mc(D)
    g = cfg['operator']['eigenvalue']
    assert rel([op.traceinv(e) for e in cfg['etas']], g['traceinv']) < 1e-9
    assert rel([op.traceinv(e, 2) for e in cfg['etas']], g['traceinv_exp2']) < 1e-9
    # exponents 1 and 2 by selected inversion and its eta-tangent: no eigenvalues
    assert op._eig is None
    assert rel([op.logdet(e) for e in cfg['etas']], g['logdet']) < 1e-9


@pytest.mark.parametrize('n', [5, 128, 129, 300, 1000])
def test_band_der_terms_vs_numpy(gp, n, monkeypatch):
    """G_p = [X z]^T (K + eta I)^-p [X z], p = 1, 2, 3, from the banded factor
    (forward, backward, forward sweeps) vs numpy, ragged n, rtol 1e-9."""
    K, X, z = _inputs(n, n + 5)
    op = _mc(K)
    etas = [1e-2, 0.3, 7.0]
    ld, G1, G2, G3 = op.der_terms(etas, X, z)
    R = numpy.column_stack([X, z])
    ref = OracleMC(K, 'cholesky')
    for i, e in enumerate(etas):
        Si = numpy.linalg.inv(K + e * numpy.eye(n))
        assert rel(ld[i], ref.logdet(e)) < 1e-10
        for G, P in ((G1, Si), (G2, Si @ Si), (G3, Si @ Si @ Si)):
            Gr = R.T @ P @ R
            numpy.testing.assert_allclose(G[i], Gr, rtol=1e-9, atol=1e-11 * numpy.abs(Gr).max())
    # the likelihood call's logdet / G1: the same sequential factorization with
    # GPMI_BAND_BCR=0 (bit for bit), by default (cyclic reduction) to rounding
    ld_l, G_l = op.loglik_terms(etas, X, z)
    assert rel(ld_l, ld) < 1e-12
    numpy.testing.assert_allclose(G_l, G1, rtol=1e-10, atol=1e-12 * numpy.abs(G1).max())
    monkeypatch.setenv('GPMI_BAND_BCR', '0')
    op0 = _mc(K)
    op0.der_terms(etas, X, z)
    ld_0, G_0 = op0.loglik_terms(etas, X, z)
    ld_d, G1_d = op0.der_terms(etas, X, z)[:2]
    numpy.testing.assert_array_equal(ld_d, ld_0)
    numpy.testing.assert_array_equal(G1_d, G_0)


def test_band_der1_der2_vs_oracle(gp):
    """ProfileLikelihood der1 (batch and scalar) and der2 on the eigenvalue
    operator (band Gram blocks + eigenvalue traces) vs the oracle's restatement
    of the reference formulas."""
    from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood
    from oracle import likelihood as olik
    K, X, z = _inputs(700, 31, nu=2.5, scale=0.1)
    op = _mc(K)
    ref = OracleMC(K, 'cholesky')
    log_etas = numpy.linspace(-3, 2, 11)
    d1 = ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, op, log_etas)
    d1_ref = [olik.profile_der1_eta(z, X, ref, le) for le in log_etas]
    assert rel(d1, d1_ref) < 1e-8
    assert rel(ProfileLikelihood.log_likelihood_der1_eta(z, X, op, -1.0),
               olik.profile_der1_eta(z, X, ref, -1.0)) < 1e-8
    for eta in (0.01, 1.0):
        assert rel(ProfileLikelihood.log_likelihood_der2_eta(z, X, op, eta),
                   olik.profile_der2_eta(z, X, ref, eta)) < 1e-7
    with pytest.raises(NotImplementedError):
        from gaussian_proc._mixed_correlation import MixedCorrelation
        MixedCorrelation(K, imate_method='cholesky').der_terms([1.0], X, z)


def test_band_der1_cfg2_golden(gp):
    """N=4096: der1 / der2 of the reference's eigenvalue operator (golden)."""
    from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood
    cfg = load_json('cfg2.json')
    pts, z, X = config_inputs(cfg)
    D = gp.generate_correlation(pts, 0.1, 1.5, device_resident=True)
    op = _mc(D)
    d1 = ProfileLikelihood.log_likelihood_der1_eta_batch(z, X, op, cfg['log_etas'])
    assert rel(d1, cfg['profile_der1_eta']) < 1e-7
    assert rel([ProfileLikelihood.log_likelihood_der2_eta(z, X, op, e)
                for e in cfg['profile_der2_eta_etas']], cfg['profile_der2_eta']) < 1e-6


def test_band_direct_jac_hess_vs_oracle(gp):
    """DirectLikelihood Jacobian / Hessian on the eigenvalue operator (band Gram
    blocks, no dense solve) vs the oracle's reference formulas; the sigma ~ 0
    branch still takes the reference path."""
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    from oracle import likelihood as olik
    K, X, z = _inputs(500, 41, nu=1.5, scale=0.15)
    op = _mc(K)
    ref = OracleMC(K, 'cholesky')
    for h in ([0.8, 0.1], [1.5, 1.2], [0.3, 1.0], [1e-9, 0.4]):
        assert rel(DirectLikelihood.log_likelihood_jacobian(z, X, op, False, h),
                   olik.direct_jac(z, X, ref, h)) < 1e-8
        if h[0] >= 1e-8:   # the reference's own Hessian formula cancels at eta ~ 1e17
            assert rel(DirectLikelihood.log_likelihood_hessian(z, X, op, True, h),
                       -olik.direct_hess(z, X, ref, h)) < 1e-7


@pytest.mark.slow
def test_band_past_single_launch_panel_limit(gp, monkeypatch):
    """n = 16640: the first panel has 129 row blocks, past the single-launch
    Householder panel QR (<= 128 workgroups): the CholeskyQR panel (default)
    and, with GPMI_BAND_PANEL=hh, the per-column hh_col path; logdet and the
    Gram block vs the dense device Cholesky (an independent factorization)."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    n = 16640
    rng = numpy.random.RandomState(7)
    pts = rng.rand(n, 2)
    D = gp.generate_correlation(pts, 0.05, 1.5, device_resident=True, max_batch=2)
    X = numpy.column_stack([numpy.ones(n), pts])
    z = numpy.cos(4 * pts[:, 1]) + 0.1 * rng.randn(n)
    etas = [0.05, 2.0]
    ld_c, G_c = MixedCorrelation(D, imate_method='cholesky').loglik_terms(etas, X, z)
    for panel in ('cholqr', 'hh'):
        if panel == 'hh':
            monkeypatch.setenv('GPMI_BAND_PANEL', 'hh')
        op = MixedCorrelation(D, imate_method='eigenvalue')
        ld_b, G_b = op.loglik_terms(etas, X, z)
        # scattered points: a numerically rank-deficient panel falls back alone
        # (the first panel, past the single-launch Householder size, by per-column
        # launches after a host check; the others by the guarded panel), and the
        # reduction runs once
        st = op.band().stats()
        print(panel, st)
        assert st['panel_fallbacks'] == 0, st
        if panel == 'cholqr':
            assert st['cholqr_fallbacks'] == 0, st
            assert st['cholqr_panel_fallbacks'] <= 8, st
        assert rel(ld_b, ld_c) < 1e-10, panel
        numpy.testing.assert_allclose(G_b, G_c, rtol=1e-8, atol=1e-10 * numpy.abs(G_c).max())


def test_band_refresh_with_rhs_matches_set_rhs(gp):
    """Q^T [X z] applied during the reduction (third stream) equals the separate
    set_rhs pass bit for bit (same kernels, same order)."""
    K, X, z = _inputs(900, 77)
    op = _mc(K)
    etas = [1e-3, 0.2, 3.0]
    ld0, G0 = op.loglik_terms(etas, X, z)
    op.refresh_band(X, z)
    ld1, G1 = op.loglik_terms(etas, X, z)
    numpy.testing.assert_array_equal(ld0, ld1)
    numpy.testing.assert_array_equal(G0, G1)
    op.refresh_band()
    ld2, G2 = op.loglik_terms(etas, X, z)
    numpy.testing.assert_array_equal(G0, G2)


def test_panel_timeout_falls_back_to_per_column_launches(gp, monkeypatch):
    """With Householder panels (GPMI_BAND_PANEL=hh), GPMI_HH_SPIN_LIMIT=0 turns the
    first unsuccessful hand-off poll of the single-launch panel QR into a timeout (as when its workgroups cannot all be
    resident): the reduction is redone with per-column launches, the result is
    the same band form, and a later refresh starts clean (err flag reset)."""
    monkeypatch.setenv('GPMI_BAND_PANEL', 'hh')   # the Householder panel
    K, X, z = _inputs(1000, 77)
    ref = _mc(K)
    ld_ref, G_ref = ref.loglik_terms([0.05, 2.0], X, z)
    assert ref.band().stats()['panel'] == 'householder'
    assert ref.band().stats()['panel_fallbacks'] == 0
    assert ref.band().stats()['panel_maxg'] >= 8
    monkeypatch.setenv('GPMI_HH_SPIN_LIMIT', '0')
    op = _mc(K)
    ld, G = op.loglik_terms([0.05, 2.0], X, z)
    st = op.band().stats()
    assert st['panel_fallbacks'] >= 1, st
    assert rel(ld, ld_ref) < 1e-12
    numpy.testing.assert_allclose(G, G_ref, rtol=1e-10, atol=1e-12)
    op.refresh_band(X, z)
    ld2, G2 = op.loglik_terms([0.05, 2.0], X, z)
    assert rel(ld2, ld_ref) < 1e-12
    assert op.band().stats()['panel_fallbacks'] >= 2


@pytest.mark.slow
def test_cfg3_nu25_n16384_dense_and_band_vs_reference(gp):
    """BASELINE cfg3 as specified (N=16384 2D grid, nu=2.5) against the
    reference's own values (tests/golden/cfg3_nu25.json, 'cholesky' imate
    method): logdet <= 1e-9 and direct lp <= 1e-8 relative, on the dense
    Cholesky operator and on the eigenvalue (band) operator."""
    from oracle import data
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    cfg = load_json('cfg3_nu25.json')
    assert cfg['nu'] == 2.5 and cfg['n'] == 16384
    pts = data.generate_points(128, 2, True)
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    D = gp.generate_correlation(pts, 0.1, 2.5, device_resident=True, max_batch=3)
    dense = MixedCorrelation(D)
    band = MixedCorrelation(D, imate_method='eigenvalue')
    for op in (dense, band):
        ld, _ = op.loglik_terms(cfg['etas'], X, z)
        assert rel(ld, cfg['logdet']) < 1e-9, op.imate_method
        lp = DirectLikelihood.log_likelihood_batch(z, X, op, cfg['hypers'])
        assert rel(lp, cfg['direct_lp']) < 1e-8, op.imate_method


@pytest.mark.parametrize('n', [129, 300, 1000, 2304])
def test_cholqr_panel_matches_householder_panel(gp, n, monkeypatch):
    """The CholeskyQR panel (shifted CholeskyQR3 + Householder reconstruction,
    gpmi_cholqr.hip; the default) and the Householder panel give the same band
    reduction up to rounding: logdet, the Gram blocks and the spectrum."""
    K, X, z = _inputs(n, 3 * n, nu=2.5)
    etas = [1e-3, 0.05, 2.0]
    op = _mc(K)
    ld, G = op.loglik_terms(etas, X, z)
    st = op.band().stats()
    assert st['panel'] == 'cholqr' and st['cholqr_fallbacks'] == 0, st
    assert st['cholqr_panel_fallbacks'] == 0, st
    monkeypatch.setenv('GPMI_BAND_PANEL', 'hh')
    oh = _mc(K)
    ld_h, G_h = oh.loglik_terms(etas, X, z)
    assert oh.band().stats()['panel'] == 'householder'
    assert rel(ld, ld_h) < 1e-12
    numpy.testing.assert_allclose(G, G_h, rtol=1e-9, atol=1e-11 * numpy.abs(G_h).max())
    lam = numpy.linalg.eigvalsh(op.band().band())
    lam_h = numpy.linalg.eigvalsh(oh.band().band())
    assert numpy.max(numpy.abs(lam - lam_h)) <= 1e-12 * numpy.abs(lam_h).max()


def test_cholqr_breakdown_falls_back_to_householder(gp):
    """A rank-deficient panel (K = I + a rank-one block: the first panel has rank
    one) breaks the CholeskyQR passes down before anything is written to it; the
    guarded Householder panel factors it on the device (no second reduction) and
    the values stay exact."""
    n = 700
    rng = numpy.random.RandomState(5)
    u = numpy.zeros(n)
    u[:200] = rng.rand(200)
    K = numpy.eye(n) + numpy.outer(u, u)
    R = numpy.column_stack([numpy.ones(n), rng.randn(n)])
    op = _mc(K)
    etas = [0.1, 1.0]
    ld, G = op.loglik_terms(etas, R[:, :1], R[:, 1])
    st = op.band().stats()
    assert st['cholqr_panel_fallbacks'] >= 1 and st['cholqr_fallbacks'] == 0, st
    for e, l, g in zip(etas, ld, G):
        M = K + e * numpy.eye(n)
        assert rel(l, numpy.linalg.slogdet(M)[1]) < 1e-12
        numpy.testing.assert_allclose(g, R.T @ numpy.linalg.solve(M, R), rtol=1e-10)


@pytest.mark.parametrize('nu', [0.5, 100.0])
def test_band_rough_and_gaussian_kernels(gp, nu):
    """Matern 1/2 (rough) and the Gaussian limit (nu >= 100: smooth, numerically
    low-rank panels, where CholeskyQR may fall back): logdet and Gram vs the
    oracle whichever panel ran."""
    K, X, z = _inputs(1000, 11, nu=nu)
    op = _mc(K)
    ref = OracleMC(K, 'cholesky')
    R = numpy.column_stack([X, z])
    for e in (0.05, 1.0):
        ld, G = op.loglik_terms([e], X, z)
        assert rel(ld[0], ref.logdet(e)) < 1e-10, (nu, e)
        numpy.testing.assert_allclose(G[0], R.T @ ref.solve(e, R), rtol=1e-7, atol=1e-9)


@pytest.mark.slow
def test_cholqr_breakdown_past_single_launch_panel_falls_back_per_panel(gp):
    """n = 16640 (the first panel has 129 row blocks, past the guarded single-launch
    Householder panel) with a rank-one first panel: the host reads that panel's
    breakdown flag after its CholeskyQR chain and factors it alone by per-column
    Householder launches; the reduction is not redone, and the values stay exact
    (K = I + u u^T: logdet = log(1 + eta + |u|^2) + (n - 1) log(1 + eta))."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    n = 16640
    rng = numpy.random.RandomState(9)
    u = numpy.zeros(n)
    u[:300] = rng.rand(300)
    K = numpy.eye(n) + numpy.outer(u, u)
    op = MixedCorrelation(K, imate_method='eigenvalue')
    etas = [0.1, 2.0]
    X = numpy.ones((n, 1))
    z = rng.randn(n)
    ld, _ = op.loglik_terms(etas, X, z)
    st = op.band().stats()
    assert st['cholqr_fallbacks'] == 0 and st['panel_fallbacks'] == 0, st
    assert st['cholqr_panel_fallbacks'] >= 1, st
    uu = u @ u
    for e, l in zip(etas, ld):
        assert rel(l, numpy.log(1 + e + uu) + (n - 1) * numpy.log(1 + e)) < 1e-12


def test_band_reduction_variants_agree(gp, monkeypatch):
    """The default reduction (CholeskyQR panels with first-order passes, look-ahead
    with the capped SYR2K grid) equals the one without look-ahead bit for bit (same
    kernels, same summation orders; only the overlap differs) and the one with an
    exact Cholesky in every pass (GPMI_CQ_FO=0) to rounding."""
    K, X, z = _inputs(2304, 41, nu=1.5, scale=0.1)
    etas = [1e-3, 0.1, 10.0]
    ld0, G0 = _mc(K).loglik_terms(etas, X, z)
    monkeypatch.setenv('GPMI_BAND_LA', '0')
    ld1, G1 = _mc(K).loglik_terms(etas, X, z)
    numpy.testing.assert_array_equal(ld0, ld1)
    numpy.testing.assert_array_equal(G0, G1)
    monkeypatch.delenv('GPMI_BAND_LA')
    monkeypatch.setenv('GPMI_CQ_FO', '0')
    ld2, G2 = _mc(K).loglik_terms(etas, X, z)
    assert rel(ld0, ld2) < 1e-12
    numpy.testing.assert_allclose(G0, G2, rtol=1e-9, atol=1e-11 * numpy.abs(G2).max())


@pytest.mark.parametrize('n', [4224, 6016])
def test_band_filler_tiles_bit_identical(gp, monkeypatch, n):
    """Sizes whose first panels' look-ahead SYR2K has more tiles than its main launch
    has workgroups (mt (mt - 1) / 2 > CUs - 32), so the tiles after the first go out
    by ticket and the filler launch after the chain takes its share: the reduction
    must still equal the one without look-ahead bit for bit (every tile updated
    exactly once, by the same product)."""
    K, X, z = _inputs(n, 7 * n + 1, nu=1.5, scale=0.1)
    etas = [1e-2, 1.0]
    ld0, G0 = _mc(K).loglik_terms(etas, X, z)
    # the look-ahead form copies only tile column 0 of K (the first panel's update reads
    # K): with the rest of the working matrix NaN beforehand, nothing may change
    monkeypatch.setenv('GPMI_BAND_POISON', '1')
    ldp, Gp = _mc(K).loglik_terms(etas, X, z)
    numpy.testing.assert_array_equal(ld0, ldp)
    numpy.testing.assert_array_equal(G0, Gp)
    monkeypatch.delenv('GPMI_BAND_POISON')
    monkeypatch.setenv('GPMI_BAND_LA', '0')
    ld1, G1 = _mc(K).loglik_terms(etas, X, z)
    numpy.testing.assert_array_equal(ld0, ld1)
    numpy.testing.assert_array_equal(G0, G1)


@pytest.mark.parametrize('n', [1, 5, 127, 128, 129, 300, 1000, 2304, 4224])
def test_band_cyclic_reduction_matches_sequential(gp, monkeypatch, n):
    """The banded Cholesky by block cyclic reduction (gpmi_bcr.hip, the default up
    to 64 eta per call: odd blocks eliminated independently per level) against the
    sequential band_chol_kernel (GPMI_BAND_BCR=0) on the same band: logdet and Gram blocks to
    rounding, for 1, 3 and 8 eta per call (levels with odd and even block counts)."""
    K, X, z = _inputs(n, 17 * n + 3, nu=1.5, scale=0.1)
    etas = [1e-3, 0.1, 2.0, 5.0, 0.02, 30.0, 0.5, 1e-2]
    monkeypatch.setenv('GPMI_BAND_BCR', '0')
    op0 = _mc(K)
    ld0, G0 = op0.loglik_terms(etas, X, z)
    monkeypatch.setenv('GPMI_BAND_BCR', '1')
    op1 = _mc(K)
    for sel in ([1], [0, 3, 5], list(range(8))):
        ld1, G1 = op1.loglik_terms([etas[i] for i in sel], X, z)
        assert rel(ld1, ld0[sel]) < 1e-12, (n, sel)
        numpy.testing.assert_allclose(G1, G0[sel], rtol=1e-9,
                                      atol=1e-11 * numpy.abs(G0).max())


def test_band_cyclic_reduction_not_spd(gp, monkeypatch):
    """An eta that leaves B + eta I indefinite raises LinAlgError through the
    cyclic reduction as through the sequential path."""
    K, X, z = _inputs(700, 5, nu=1.5, scale=0.2)
    lam = numpy.linalg.eigvalsh(K)
    monkeypatch.setenv('GPMI_BAND_BCR', '1')
    op = _mc(K)
    with pytest.raises(numpy.linalg.LinAlgError):
        op.loglik_terms([0.1, -lam[0] - 0.5 * (lam[1] - lam[0]) - 1e-3], X, z)


@pytest.mark.parametrize('n', [1, 5, 128, 129, 300, 1000, 2177])
def test_band_selected_inversion_traceinv(gp, n):
    """trace((K + eta I)^-1) by selected inversion of the cyclic-reduction factor
    down its reduction tree (gpmi_band_traceinv, no eigenvalues) vs numpy's
    eigenvalue sums at ragged n (1 to 18 blocks, odd and even level sizes), rel
    <= 1e-10; the same numbers from der_terms(traceinv=True) (one factorization
    for the Gram blocks and the trace) and, once computed, from the device
    eigenvalues."""
    K, X, z = _inputs(n, n + 11, nu=2.5, scale=0.15)
    lam = numpy.linalg.eigvalsh(K)
    etas = numpy.array([1e-3, 0.05, 1.0, 30.0])
    exact = numpy.array([numpy.sum(1.0 / (lam + e)) for e in etas])
    op = _mc(K)
    tr, info = op.band().traceinv(etas)
    assert not numpy.any(info)
    assert rel(tr, exact) < 1e-10, (tr, exact)
    ld, G1, G2, G3, tr1 = op.der_terms(etas, X, z, traceinv=True)
    assert rel(tr1, tr) < 1e-12
    # MixedCorrelation.traceinv(eta) answers by selected inversion first
    assert op._eig is None
    assert rel(op.traceinv(0.05), exact[1]) < 1e-10 and op._eig is None
    lam_d = op.eigenvalues()
    assert rel(numpy.sum(1.0 / (lam_d + 0.05)), tr[1]) < 1e-10
    # with the eigenvalues cached, der_terms takes its traces from them
    tr1e = op.der_terms(etas[:2], X, z, traceinv=True)[4]
    assert rel(tr1e, tr[:2]) < 1e-10


def test_band_selected_inversion_not_spd_and_many_etas(gp):
    """A non-SPD shift reports its pivot through the band's selected inversion;
    MixedCorrelation.traceinv then answers from the eigenvalue sums, as the
    reference's eigenvalue traceinv (which never raises) does, for exponents 1 and
    2 alike. 150 etas in one call (three cyclic-reduction chunks of <= 64) equal
    the per-eta values, for both exponents."""
    K, X, z = _inputs(600, 77)
    lam = numpy.linalg.eigvalsh(K)
    op = _mc(K)
    bad = -lam[0] - 1.0
    for p in (1, 2):
        tr, info = op.band().traceinv([bad], p)
        assert info[0] > 0
    assert op._eig is None
    for p in (1, 2):
        assert rel(op.traceinv(bad, p), numpy.sum((lam + bad) ** -float(p))) < 1e-9
    etas = numpy.logspace(-2, 2, 150)
    for p in (1, 2):
        tr, info = op.band().traceinv(etas, p)
        assert not numpy.any(info)
        exact = numpy.array([numpy.sum((lam + e) ** -float(p)) for e in etas])
        assert rel(tr, exact) < 1e-10, p


@pytest.mark.parametrize('n', [1, 5, 128, 129, 300, 1000, 2177])
def test_band_selected_inversion_traceinv_exponent_2(gp, n):
    """trace((K + eta I)^-2) as -d/deta trace((K + eta I)^-1): the cyclic-reduction
    factor and its selected inversion differentiated in eta in forward mode
    (gpmi_band_traceinv2, no eigenvalues) vs numpy's eigenvalue sums at ragged n,
    rel <= 1e-10; the same numbers from der_terms(traceinv=2) (one factorization
    for the Gram blocks and both traces) and MixedCorrelation.traceinv(eta, 2)
    without the eigenvalue chase."""
    K, X, z = _inputs(n, n + 17, nu=2.5, scale=0.15)
    lam = numpy.linalg.eigvalsh(K)
    etas = numpy.array([1e-3, 0.05, 1.0, 30.0])
    ex1 = numpy.array([numpy.sum(1.0 / (lam + e)) for e in etas])
    ex2 = numpy.array([numpy.sum((lam + e) ** -2.0) for e in etas])
    op = _mc(K)
    tr2, info = op.band().traceinv(etas, 2)
    assert not numpy.any(info)
    assert rel(tr2, ex2) < 1e-10, (tr2, ex2)
    ld, G1, G2, G3, tr1d, tr2d = op.der_terms(etas, X, z, traceinv=2)
    assert rel(tr1d, ex1) < 1e-10 and rel(tr2d, tr2) < 1e-12
    # the Gram blocks of the tangent-carrying call equal the plain call's
    ld0, G10, G20, G30, info0 = op.band().der_terms(etas)
    assert rel(ld, ld0) < 1e-13 and rel(G2, G20) < 1e-12 and rel(G3, G30) < 1e-12
    assert rel(op.traceinv(0.05, 2), ex2[1]) < 1e-10
    assert op._eig is None
