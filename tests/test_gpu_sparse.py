"""Sparse (tapered Matérn) path on an MI355X vs the reference fixtures and the
oracle: CSR assembly (reference + 2 argument fixes), SpMM, Lanczos / SLQ with
identical counter-based probes, blocked CG, and the sparse likelihood.

Tolerances: CSR structure bit-exact, values <= 4e-16 abs; Lanczos coefficients
and SLQ sums vs the oracle with the same probes <= 1e-9 relative; SLQ vs exact
within Monte-Carlo error; CG solutions <= 1e-5 relative (reference rtol 1e-6).
"""

import numpy
import pytest
import scipy.sparse.linalg

from oracle import data, sparse as osp
from oracle import likelihood as olk
from _util import load_json, load_npz, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def gp():
    import gaussian_proc
    from gaussian_proc import _hip
    _hip.require_device(0)
    return gaussian_proc


@pytest.mark.parametrize('case', [0, 1, 2])
def test_sparse_assembly_matches_reference(gp, case):
    meta = load_json('sparse.json')[case]
    arr = load_npz('sparse_small.npz')
    pts = data.generate_points(meta['num_points'], meta['dimension'], True)
    K = gp.generate_correlation(pts, meta['correlation_scale'], meta['nu'], sparse=True,
                                density=meta['density'])
    name = meta['name']
    numpy.testing.assert_array_equal(K.indptr, arr[name + '_indptr'])
    numpy.testing.assert_array_equal(K.indices, arr[name + '_indices'])
    assert numpy.max(numpy.abs(K.data - arr[name + '_data'])) <= 4e-16
    assert K.nnz == meta['nnz']


def test_sparse_config4_nnz_matches_reference(gp):
    meta = [m for m in load_json('sparse.json') if m['name'] == 'sp2d_n65536_cfg4'][0]
    pts = data.generate_points(256, 2, True)
    D = gp.generate_correlation(pts, 0.005, 1.5, sparse=True, density=1e-3,
                                device_resident=True)
    assert D.nnz == meta['nnz']
    K = D.tocsr()
    assert abs(K.data.sum() - meta['data_sum']) <= 1e-12 * meta['data_sum']
    assert K.data.min() == pytest.approx(meta['min_kept'], rel=1e-15)


def test_threshold_error_matches_reference(gp):
    pts = data.generate_points(10, 2, True)
    with pytest.raises(ValueError):
        gp.generate_correlation(pts, 0.1, 1.5, sparse=True, density=1e-3)


def _small_sparse():
    pts = data.generate_points(24, 2, True)
    K, tau = osp.sparse_correlation(pts, 0.08, 1.5, 0.03)
    return pts, K


def test_spmm_and_cg(gp):
    from gaussian_proc import _hip
    _, K = _small_sparse()
    sop = _hip.SparseOperator.from_csr(K)
    rng = numpy.random.RandomState(0)
    X = rng.randn(K.shape[0], 5)
    numpy.testing.assert_allclose(sop.spmm(0.7, X), K @ X + 0.7 * X, rtol=1e-13, atol=1e-13)
    eta = 3.0   # > |lambda_min| of the (indefinite) tapered matrix
    A = (K + eta * scipy.sparse.eye(K.shape[0])).tocsc()
    Y = sop.cg(eta, X, rtol=1e-10)
    numpy.testing.assert_allclose(Y, scipy.sparse.linalg.spsolve(A, X), rtol=1e-8, atol=1e-9)


def _nrel(a, b):
    return float(numpy.max(numpy.abs(a - b)) / numpy.max(numpy.abs(b)))


def test_multishift_gram_vs_exact(gp):
    """One multi-shift CG on K + min(eta) I gives B^T (K + eta I)^-1 B for every
    eta; vs scipy's sparse direct solve (Gram error is quadratic in the CG
    residual: rel <= 1e-9 at rtol 1e-8, <= 1e-6 at the reference's 1e-6)."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    n = K.shape[0]
    sop = _hip.SparseOperator.from_csr(K)
    rng = numpy.random.RandomState(5)
    B = rng.randn(n, 7)
    etas = numpy.array([10.0, 2.5, 4.0, 100.0])
    for rtol, tol in ((1e-8, 1e-9), (1e-6, 1e-6)):
        G = sop.msgram(etas, B, rtol=rtol)
        for e, g in zip(etas, G):
            A = (K + e * scipy.sparse.eye(n)).tocsc()
            ex = B.T @ scipy.sparse.linalg.spsolve(A, B)
            assert _nrel(g, ex) < tol, (rtol, e)
    # 11 columns (3D degree-2 basis + z) and a 1-column RHS
    B11 = rng.randn(n, 11)
    G = sop.msgram([3.0], B11, rtol=1e-10)
    ex = B11.T @ scipy.sparse.linalg.spsolve((K + 3.0 * scipy.sparse.eye(n)).tocsc(), B11)
    assert _nrel(G[0], ex) < 1e-10
    g1 = sop.msgram([3.0, 7.0], B[:, 0], rtol=1e-10)
    assert g1.shape == (2, 1, 1)


def test_lanczos_and_slq_match_oracle_same_probes(gp):
    from gaussian_proc import _hip, _slq
    _, K = _small_sparse()
    n = K.shape[0]
    sop = _hip.SparseOperator.from_csr(K)
    nprobe, steps, seed = 6, 25, 11
    a, b = sop.lanczos(nprobe, steps, seed)
    P = osp.rademacher_probes(n, nprobe, seed)
    for p in range(nprobe):
        ao, bo = osp.lanczos(K, P[:, p], steps)
        k = ao.size
        assert rel(a[p, :k], ao) < 1e-9
        assert rel(b[p, :k - 1], bo) < 1e-9
    etas = [2.5, 10.0]
    ref = osp.slq(K, etas, P, steps)
    nodes = _slq.nodes(a, b)
    for what in ('logdet', 'traceinv', 'traceinv2'):
        est = n * _slq.quadrature(nodes, etas, _slq.FUNCS[what]).mean(axis=0)
        assert rel(est, ref[what]) < 1e-9, what


def test_sparse_operator_slq_vs_exact(gp):
    from gaussian_proc._mixed_correlation import MixedCorrelation
    _, K = _small_sparse()
    n = K.shape[0]
    op = MixedCorrelation(K, imate_method='slq',
                          imate_options={'num_samples': 64, 'lanczos_degree': 30})
    Kd = K.toarray()
    for eta in (2.5, 10.0):
        ex = numpy.linalg.slogdet(Kd + eta * numpy.eye(n))[1]
        assert abs(op.logdet(eta) - ex) < 0.01 * abs(ex) + 1.0
        exi = numpy.trace(numpy.linalg.inv(Kd + eta * numpy.eye(n)))
        assert abs(op.traceinv(eta) - exi) < 0.03 * exi
    hop = MixedCorrelation(K, imate_method='hutchinson', imate_options={'num_samples': 64})
    exi = numpy.trace(numpy.linalg.inv(Kd + 5.0 * numpy.eye(n)))
    assert abs(hop.traceinv(5.0) - exi) < 0.05 * exi
    with pytest.raises(NotImplementedError):
        MixedCorrelation(K, imate_method='cholesky').logdet(5.0)
    # trace / dot use the CSR exactly
    assert rel(op.trace(0.5, 2), numpy.trace((Kd + 0.5 * numpy.eye(n)) @
                                            (Kd + 0.5 * numpy.eye(n)))) < 1e-12
    x = numpy.arange(n, dtype=float)
    numpy.testing.assert_allclose(op.dot(0.5, x, 2), 2 * (Kd @ x + 0.5 * x), rtol=1e-13)


def test_sparse_likelihood_vs_oracle(gp):
    """Direct lp with a sparse K: SLQ logdet + CG solves vs the oracle's exact
    lp (dense) within the SLQ Monte-Carlo error."""
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from oracle.mixed_correlation import MixedCorrelation as OracleMC
    pts, K = _small_sparse()
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    op = MixedCorrelation(K, imate_method='slq',
                          imate_options={'num_samples': 64, 'lanczos_degree': 30})
    ref = OracleMC(K.toarray(), 'cholesky')
    for hp in ([1.0, 2.0], [0.5, 1.5]):
        lp = DirectLikelihood.log_likelihood(z, X, op, False, hp)
        lp_ref = olk.direct_lp(z, X, ref, hp)
        assert abs(lp - lp_ref) < 0.01 * abs(lp_ref) + 1.0


@pytest.mark.parametrize('dim,npts,rho,dens', [(1, 3000, 0.01, 1e-2), (2, 2500, 0.02, 5e-3),
                                               (3, 4096, 0.03, 4e-3)])
def test_cell_list_assembly_equals_all_pairs(gp, monkeypatch, dim, npts, rho, dens):
    """The cell-list CSR (default for d <= 3) is bit-identical to the all-pairs
    kernels on scattered (non-grid) points, ragged cell occupancy included."""
    rng = numpy.random.RandomState(7 + dim)
    pts = rng.rand(npts, dim)
    pts[:7] = pts[0]                     # coincident points share a cell
    K = gp.generate_correlation(pts, rho, 1.5, grid=False, sparse=True, density=dens)
    monkeypatch.setenv('GPMI_SPARSE_BRUTE', '1')
    B = gp.generate_correlation(pts, rho, 1.5, grid=False, sparse=True, density=dens)
    numpy.testing.assert_array_equal(K.indptr, B.indptr)
    numpy.testing.assert_array_equal(K.indices, B.indices)
    numpy.testing.assert_array_equal(K.data, B.data)
    assert K.nnz > npts
