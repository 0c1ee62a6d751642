"""Pin the CPU oracle (oracle/) against the golden vectors produced by the
reference itself (tests/golden/make_golden.py) — CPU only."""

import numpy
import pytest

from oracle import data, matern, likelihood as olk
from oracle.mixed_correlation import MixedCorrelation as OracleMC
from _util import load_json, load_npz, config_inputs, rel


def test_matern_small_cases_match_reference_cython():
    meta = load_json('matern_small.json')
    arr = load_npz('matern_small.npz')
    for case in meta:
        c = case['case']
        pts = arr['points_%d' % c]
        K_ref = arr['K_%d' % c]
        K = matern.dense_correlation(pts, case['correlation_scale'], case['nu'])
        # closed forms: a few ulp; general nu (scipy kv vs same kv): tight
        assert numpy.max(numpy.abs(K - K_ref)) <= 4e-15, case
        numpy.testing.assert_array_equal(K, K.T)


@pytest.mark.parametrize('name', ['cfg1.json', 'cfg2.json', 'n1024_nu25.json'])
def test_inputs_match_reference_generators(name):
    cfg = load_json(name)
    pts, z, X = config_inputs(cfg)
    assert X.shape == (cfg['n'], cfg['m'])
    assert abs(z.sum() - cfg['z_sum']) <= 1e-12 * abs(cfg['z_sum'])
    numpy.testing.assert_allclose(z[cfg['sample_rows']], cfg['z_samples'], rtol=0, atol=0)
    numpy.testing.assert_allclose(X.sum(axis=0), cfg['X_col_sums'], rtol=1e-14)


def _oracle_ops(cfg):
    pts, z, X = config_inputs(cfg)
    K = matern.dense_correlation(pts, cfg['correlation_scale'], cfg['nu'])
    return K, z, X


@pytest.mark.parametrize('name', ['cfg1.json', 'n1024_nu25.json'])
def test_oracle_operator_and_likelihood(name):
    cfg = load_json(name)
    K, z, X = _oracle_ops(cfg)
    assert rel(K.sum(), cfg['K_sum']) < 1e-13
    ks = cfg['K_samples']
    numpy.testing.assert_allclose(K[ks['i'], ks['j']], ks['v'], rtol=1e-14, atol=1e-16)
    chol = OracleMC(K, 'cholesky')
    eig = OracleMC(K, 'eigenvalue')
    for meth, op in (('cholesky', chol), ('eigenvalue', eig)):
        g = cfg['operator'][meth]
        assert rel([op.logdet(e) for e in cfg['etas']], g['logdet']) < 1e-10
        assert rel([op.traceinv(e) for e in cfg['etas']], g['traceinv']) < 1e-9
        assert rel([op.traceinv(e, 2) for e in cfg['etas']], g['traceinv_exp2']) < 1e-9
        for p in ('0', '1', '2'):
            assert rel([op.trace(e, int(p)) for e in [0.0] + cfg['etas']],
                       g['trace'][p]) < 1e-12
    assert rel([olk.direct_lp(z, X, chol, h) for h in cfg['hypers']],
               cfg['direct_lp']) < 1e-9
    for h, jref, href in zip(cfg['hypers'], cfg['direct_jac'], cfg['direct_hess']):
        assert rel(olk.direct_jac(z, X, chol, h), jref) < 1e-7
        if h[0] < 1e-8:
            # sigma = 1e-9 takes the eta = 9e16 branch of the Hessian (its threshold is
            # 1e-16, _direct_likelihood.py:179): the H_ss entry (~1e23) is rounding
            # noise in the reference too; compare the well-conditioned entries only.
            hh = olk.direct_hess(z, X, chol, h)
            assert rel(hh[1, 1], href[1][1]) < 1e-6
            continue
        assert rel(olk.direct_hess(z, X, chol, h), href) < 1e-6
    assert rel([olk.profile_lp(z, X, chol, h) for h in cfg['profile_hypers']],
               cfg['profile_lp']) < 1e-9
    assert rel([olk.profile_der1_eta(z, X, chol, le) for le in cfg['log_etas']],
               cfg['profile_der1_eta']) < 1e-7
    assert rel([olk.profile_der2_eta(z, X, chol, e) for e in cfg['profile_der2_eta_etas']],
               cfg['profile_der2_eta']) < 1e-6
    w = chol.solve(1.0, z)
    numpy.testing.assert_allclose(w[cfg['sample_rows']], cfg['solve_eta1_z_samples'],
                                  rtol=1e-10)
    d2 = chol.dot(0.5, z, exponent=2)
    numpy.testing.assert_allclose(d2[cfg['sample_rows']], cfg['dot_eta05_exp2_z_samples'],
                                  rtol=1e-13)


def test_oracle_cfg2_scalars():
    """N=4096 (config 2): the oracle's Cholesky path vs the reference's eigen path."""
    cfg = load_json('cfg2.json')
    K, z, X = _oracle_ops(cfg)
    assert rel(K.sum(), cfg['K_sum']) < 1e-13
    op = OracleMC(K, 'cholesky')
    assert rel([op.logdet(e) for e in cfg['etas']], cfg['operator']['eigenvalue']['logdet']) \
        < 1e-10
    assert rel([olk.direct_lp(z, X, op, h) for h in cfg['hypers'][:2]],
               cfg['direct_lp'][:2]) < 1e-9


def test_survey_appendix_a_values():
    """Known answers recorded in SURVEY.md Appendix A (same reference, earlier run)."""
    c1 = load_json('cfg1.json')
    assert rel(c1['K_sum'], 13775.437627800122) < 1e-15
    assert rel(c1['direct_lp'][0], 44.876424215886686) < 1e-12
    assert rel(c1['operator']['eigenvalue']['logdet'],
               [-1413.1733976433375, -497.9485597428433, 39.08480792780253,
                601.7708016118943]) < 1e-12
    c2 = load_json('cfg2.json')
    assert rel(c2['direct_lp'][:2], [677.58921379509, -1228.4678497026616]) < 1e-12


def test_data_generators_shapes():
    pts = data.generate_points(5, 3, True)
    assert pts.shape == (125, 3)
    X = data.generate_basis_functions(pts, 2)
    assert X.shape == (125, 10)
