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


def _host_cg_iterations(A, B, rtol):
    """Iterations of the per-column CG gpmi_sp_cg runs (a column stops once
    ||r|| <= rtol ||b||; the count is the last iteration any column ran)."""
    its = 0
    for c in range(B.shape[1]):
        b = B[:, c]
        x = numpy.zeros_like(b)
        r = b.copy()
        p = r.copy()
        rr = r @ r
        k = 0
        while numpy.sqrt(rr) > rtol * numpy.linalg.norm(b):
            q = A @ p
            a = rr / (p @ q)
            x += a * p
            r -= a * q
            rrn = r @ r
            p = r + (rrn / rr) * p
            rr = rrn
            k += 1
        its = max(its, k)
    return its


def test_cg_device_scalars(gp):
    """gpmi_sp_cg keeps its scalars on the device (the host polls every 8
    iterations): the iteration count equals a host CG's (+-1 for rounding at the
    threshold), a zero right-hand side stays zero without stopping the others,
    and a run that stops between polls returns the converged iterate."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    sop = _hip.SparseOperator.from_csr(K)
    n = K.shape[0]
    eta = 3.0
    A = (K + eta * scipy.sparse.eye(n)).tocsr()
    B = numpy.random.RandomState(5).randn(n, 4)
    B[:, 2] = 0.0
    for rtol in (1e-4, 1e-10):
        Y = sop.cg(eta, B, rtol=rtol)
        ex = scipy.sparse.linalg.spsolve(A.tocsc(), B)
        assert numpy.all(Y[:, 2] == 0.0)
        assert _nrel(Y, ex) < 50 * rtol
        assert abs(sop.last_cg_iterations - _host_cg_iterations(A, B, rtol)) <= 1
    Y = sop.cg(eta, B[:, 2], rtol=1e-8)
    assert numpy.all(Y == 0.0) and sop.last_cg_iterations == 0


def test_window_spmm_equals_gather_spmm(gp, monkeypatch):
    """The X-window SpMM (64-row blocks, window rows staged in LDS; the default
    where its blocks fit 32 KB of LDS, e.g. 2D tapered Matern) against the
    one-wave-per-row gather kernel and scipy, for s = 1 .. 32
    columns, on a matrix whose first blocks overflow the window limits (more
    than 4096 nonzeros, more than 1024 distinct columns) and so take the
    gather path inside the same launch. For even s the gather is the column-pair
    kernel; GPMI_SPMM_PAIR=0 gives the one-column gather to compare with. At
    s = 7, 11, 20 the default is the window with latency-hidden staging
    (csr_spmm_wing_kernel); GPMI_SPMM_WING=0 gives the chunked window kernel."""
    from gaussian_proc import _hip
    rng = numpy.random.RandomState(4)
    n = 3000
    rows, cols = [], []
    for i in range(n):
        if i < 64:
            k = 100                                  # 6400 nonzeros in block 0
            c = rng.choice(n, k, replace=False)
        elif i < 128:
            c = rng.choice(n, 40, replace=False)     # ~2000 distinct columns in block 1
        else:
            c = numpy.clip(i + rng.randint(-30, 31, 12), 0, n - 1)
        rows.extend([i] * len(c))
        cols.extend(c)
    A = scipy.sparse.csr_matrix((rng.randn(len(rows)), (rows, cols)), shape=(n, n))
    A = (A + A.T).tocsr()
    A.sum_duplicates()
    A.sort_indices()
    sop = _hip.SparseOperator.from_csr(A)
    for s in (1, 7, 8, 11, 20, 32):
        X = rng.randn(n, s)
        # the window with latency-hidden staging (default at s = 7, 11, 20)
        Ywg = sop.spmm(0.3, X)
        if s in (7, 11, 20):
            assert sop.spmm_kernel(s) == 'csr_spmm_wing_kernel'
        monkeypatch.setenv('GPMI_SPMM_WING', '0')
        monkeypatch.setenv('GPMI_SPMM_WINDOW', '2')
        Yw = sop.spmm(0.3, X)
        monkeypatch.setenv('GPMI_SPMM_WINDOW', '0')
        Yg = sop.spmm(0.3, X)
        monkeypatch.setenv('GPMI_SPMM_PAIR', '0')
        Y1 = sop.spmm(0.3, X)
        assert sop.spmm_kernel(s) == 'csr_spmm_kernel'
        monkeypatch.delenv('GPMI_SPMM_PAIR')
        assert sop.spmm_kernel(s) == ('csr_spmm_pair_kernel' if s % 2 == 0 else 'csr_spmm_kernel')
        monkeypatch.delenv('GPMI_SPMM_WINDOW')
        monkeypatch.delenv('GPMI_SPMM_WING')
        ref = A @ X + 0.3 * X
        assert _nrel(Ywg, ref) < 1e-13, s
        assert _nrel(Yw, ref) < 1e-13, s
        assert _nrel(Yw, Yg) < 1e-13, s
        assert _nrel(Y1, Yg) < 1e-13, s


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


def test_msgram_column_shards_equal_full(gp):
    """gpmi_sp_msgram_cols: shards of the right-hand-side columns, each solved for
    every eta and dotted with all of B, give the columns of the full multi-shift
    Gram (the per-column CG recurrences do not depend on the other columns; the
    shards run other kernel forms, so equal to 1e-9, not bit for bit), and vs
    the exact solve."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    n = K.shape[0]
    sop = _hip.SparseOperator.from_csr(K)
    rng = numpy.random.RandomState(7)
    B = rng.randn(n, 11)
    etas = numpy.array([2.5, 4.0, 10.0, 100.0])
    G = sop.msgram(etas, B, rtol=1e-10)
    for lo, hi in ((0, 2), (2, 3), (3, 9), (9, 11), (0, 11)):
        Gc = sop.msgram(etas, B, rtol=1e-10, cols=(lo, hi))
        assert Gc.shape == (etas.size, 11, hi - lo)
        assert _nrel(Gc, G[:, :, lo:hi]) < 1e-9, (lo, hi)
    for e, g in zip(etas, G):
        ex = B.T @ scipy.sparse.linalg.spsolve((K + e * scipy.sparse.eye(n)).tocsc(), B)
        assert _nrel(g, ex) < 1e-9


def test_msgram_resident_rhs(gp):
    """gpmi_sp_set_rhs: the right-hand sides kept in HBM give the same Gram as the
    host block, bit for bit (the same kernels on the same values), for the full
    block and a column shard; a block of another width replaces it; without one,
    msgram(etas, None) raises."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    n = K.shape[0]
    sop = _hip.SparseOperator.from_csr(K)
    etas = numpy.array([3.0, 6.0, 50.0])
    with pytest.raises(ValueError):
        sop.msgram(etas, None)
    rng = numpy.random.RandomState(11)
    for s in (11, 4):
        B = rng.randn(n, s)
        G = sop.msgram(etas, B, rtol=1e-10)
        sop.set_rhs(B)
        assert numpy.array_equal(sop.msgram(etas, None, rtol=1e-10), G)
        assert numpy.array_equal(sop.msgram(etas, None, rtol=1e-10, cols=(1, 3)),
                                 sop.msgram(etas, B, rtol=1e-10, cols=(1, 3)))


def test_msgram_widths_vs_exact_solve(gp):
    """The multi-shift CG (r update and B^T r, r . r on MFMA, ms_rmfma_kernel; partial
    sums across the chip) at 3, 7 and 11 columns (11 padded to 12 on the window SpMM)
    against the exact solve's Gram."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    n = K.shape[0]
    sop = _hip.SparseOperator.from_csr(K)
    rng = numpy.random.RandomState(3)
    etas = numpy.array([2.5, 7.0, 40.0])
    for s in (3, 7, 11):
        B = rng.randn(n, s)
        G = sop.msgram(etas, B, rtol=1e-10)
        for e, g in zip(etas, G):
            ex = B.T @ scipy.sparse.linalg.spsolve((K + e * scipy.sparse.eye(n)).tocsc(), B)
            assert _nrel(g, ex) < 1e-9, (s, e)


def test_msgram_stopped_column_and_overflowing_windows(gp):
    """The multi-shift CG on the window SpMM (csr_spmm_wing_kernel at s = 7 and 11)
    over a matrix whose first blocks overflow the window (the gather branch), with a
    zero right-hand side (a column stopped from the start: its p and x stay zero):
    the Gram matches the exact solve, the zero column's row and column exactly 0."""
    from gaussian_proc import _hip
    rng = numpy.random.RandomState(5)
    n = 3000
    rows, cols = [], []
    for i in range(n):
        if i < 64:
            c = rng.choice(n, 100, replace=False)
        elif i < 128:
            c = rng.choice(n, 40, replace=False)
        else:
            c = numpy.clip(i + rng.randint(-30, 31, 12), 0, n - 1)
        rows.extend([i] * len(c))
        cols.extend(c)
    A = scipy.sparse.csr_matrix((numpy.abs(rng.randn(len(rows))), (rows, cols)), shape=(n, n))
    A = (A + A.T).tocsr()
    A.sum_duplicates()
    # symmetric, diagonally dominant: positive definite
    A = (A + scipy.sparse.diags(numpy.asarray(A.sum(axis=1)).ravel() + 0.1)).tocsr()
    A.sort_indices()
    sop = _hip.SparseOperator.from_csr(A)
    etas = numpy.array([0.5, 2.0, 30.0])
    for s in (7, 11):
        assert sop.spmm_kernel(s) == 'csr_spmm_wing_kernel'
        B = rng.randn(n, s)
        B[:, 3] = 0.0
        G = sop.msgram(etas, B, rtol=1e-11, maxiter=2000)
        assert not G[:, 3, :].any() and not G[:, :, 3].any()
        for e, g in zip(etas, G):
            ex = B.T @ scipy.sparse.linalg.spsolve((A + e * scipy.sparse.eye(n)).tocsc(), B)
            assert _nrel(g, ex) < 1e-9, (s, e)


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


def test_lanczos_without_reorthogonalisation_matches_oracle(gp):
    """imate's orthogonalize option: 0 (imate's default) is the plain three-term
    recurrence, against the oracle's (oracle.sparse.lanczos reorth=False) with the
    same probes: alpha / beta <= 1e-9 over 12 steps (before the recurrence loses
    orthogonality the two agree to rounding; later steps amplify the rounding
    differences, so the SLQ sums are compared at 1e-6); a window of 3 previous
    vectors lies between the two; -1 is the full DCGS2 path."""
    from gaussian_proc import _hip, _slq
    from gaussian_proc._mixed_correlation import MixedCorrelation
    _, K = _small_sparse()
    n = K.shape[0]
    sop = _hip.SparseOperator.from_csr(K)
    nprobe, seed = 6, 11
    P = osp.rademacher_probes(n, nprobe, seed)
    a, b = sop.lanczos(nprobe, 12, seed, orthogonalize=0)
    for p in range(nprobe):
        ao, bo = osp.lanczos(K, P[:, p], 12, reorth=False)
        k = ao.size
        assert rel(a[p, :k], ao) < 1e-9
        assert rel(b[p, :k - 1], bo) < 1e-9
    steps = 25
    a0, b0 = sop.lanczos(nprobe, steps, seed, orthogonalize=0)
    ref = osp.slq(K, [2.5, 10.0], P, steps, reorth=False)
    est = n * _slq.quadrature(_slq.nodes(a0, b0), [2.5, 10.0], numpy.log).mean(axis=0)
    assert rel(est, ref['logdet']) < 1e-6
    af, bf = sop.lanczos(nprobe, steps, seed)
    aw, bw = sop.lanczos(nprobe, steps, seed, orthogonalize=3)
    full = n * _slq.quadrature(_slq.nodes(af, bf), [2.5, 10.0], numpy.log).mean(axis=0)
    win = n * _slq.quadrature(_slq.nodes(aw, bw), [2.5, 10.0], numpy.log).mean(axis=0)
    # every variant estimates the same logdet (Monte-Carlo error of 6 probes >> these)
    assert rel(win, full) < 1e-3 and rel(est, full) < 1e-3
    op = MixedCorrelation(K, imate_method='slq',
                          imate_options={'num_samples': nprobe, 'lanczos_degree': steps,
                                         'seed': seed, 'orthogonalize': 0})
    assert op.logdet(2.5) == pytest.approx(est[0], rel=1e-12)


def test_slq_adaptive_sample_count(gp):
    """imate's adaptive sampling (min_num_samples / max_num_samples / error_rtol /
    confidence_level): probes are added until the confidence half width meets the
    tolerance; the estimate equals the fixed-count one at the count it stopped at
    (counter-based probes: a prefix of the same probe set)."""
    import scipy.stats
    from gaussian_proc._mixed_correlation import MixedCorrelation
    _, K = _small_sparse()
    opts = {'min_num_samples': 4, 'max_num_samples': 40, 'error_rtol': 2e-3,
            'lanczos_degree': 25, 'seed': 5}
    op = MixedCorrelation(K, imate_method='slq', imate_options=opts)
    v = op.logdet(2.5)
    k = op.last_num_samples
    assert 4 <= k <= 40
    # the adaptive probes are kept apart: the fixed set (num_samples, slq_nodes)
    # does not grow with earlier calls, and a repeat call gives the same value
    assert op.num_samples == 4 and len(op.slq_nodes()) == 4
    assert op.logdet(2.5) == v and op.last_num_samples == k
    fixed = MixedCorrelation(K, imate_method='slq',
                             imate_options={'num_samples': k, 'lanczos_degree': 25, 'seed': 5})
    assert v == pytest.approx(fixed.logdet(2.5), rel=1e-12)
    q = numpy.array([K.shape[0] * numpy.sum(w * numpy.log(t + 2.5))
                     for t, w in fixed.slq_nodes()])
    half = scipy.stats.norm.ppf(0.975) * q.std(ddof=1) / numpy.sqrt(q.size)
    assert k == 40 or half <= 2e-3 * abs(q.mean())
    # a looser tolerance stops at the minimum
    op2 = MixedCorrelation(K, imate_method='slq',
                           imate_options={'min_num_samples': 4, 'error_rtol': 0.5,
                                          'lanczos_degree': 25})
    op2.logdet(2.5)
    assert op2.last_num_samples == 4


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
    # trace / dot use the CSR exactly
    assert rel(op.trace(0.5, 2), numpy.trace((Kd + 0.5 * numpy.eye(n)) @
                                            (Kd + 0.5 * numpy.eye(n)))) < 1e-12
    x = numpy.arange(n, dtype=float)
    numpy.testing.assert_allclose(op.dot(0.5, x, 2), 2 * (Kd @ x + 0.5 * x), rtol=1e-13)


def test_sparse_slq_lanczos_tol_converges(gp):
    """imate's lanczos_tol on a SPARSE (tapered, indefinite) K: the Gauss-Radau
    node is the smallest Ritz value minus a margin (the Gershgorin bound lies
    below -eta, where log is NaN: ADVICE r4), so the bracket closes at a
    moderate tolerance instead of running to max_lanczos_degree unconverged;
    the logdet stays within 4 probe standard errors of the exact value."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    pts = data.generate_points(24, 2, True)
    K, _ = osp.sparse_correlation(pts, 0.08, 1.5, 0.1)   # Gershgorin -9.3, lambda_min -0.79
    n = K.shape[0]
    Kd = K.toarray()
    lam = numpy.linalg.eigvalsh(Kd)
    op = MixedCorrelation(K, imate_method='slq',
                          imate_options={'num_samples': 48, 'lanczos_degree': 8,
                                         'lanczos_tol': 1e-7})
    assert op._lower_bound() + 5.0 < 0.0     # the Gershgorin bound is useless here
    for eta in (1.5, 5.0):
        val = op.logdet(eta)
        conv = op.last_slq_convergence
        assert conv['converged'] and conv['bracket'] <= 1e-7, conv
        assert conv['degree'] < op.max_lanczos_degree and not conv['rigorous_bound'], conv
        assert conv['radau_node'] + eta > 0.0
        ex = float(numpy.sum(numpy.log(lam + eta)))
        q = n * _slq_probe_values(op, eta)
        se = q.std(ddof=1) / numpy.sqrt(q.size)
        assert abs(val - ex) < 4 * se + 1e-9 * abs(ex), (eta, val, ex, se)


def _slq_probe_values(op, eta):
    from gaussian_proc import _slq
    return _slq.quadrature(op.slq_nodes(), [eta], numpy.log)[:, 0]


def test_sparse_hutchinson_traceinv_exponent_3(gp):
    """Sparse 'hutchinson' traceinv of exponent 3: two chained device CG solves
    per probe (rtol 1e-10 here), within 4 standard errors of the eigenvalue sum."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    _, K = _small_sparse()
    n = K.shape[0]
    Kd = K.toarray()
    lam = numpy.linalg.eigvalsh(Kd)
    s = 64
    hop = MixedCorrelation(K, imate_method='hutchinson',
                           imate_options={'num_samples': s, 'cg_rtol': 1e-10})
    for eta in (5.0, 10.0):
        B = numpy.linalg.matrix_power(numpy.linalg.inv(Kd + eta * numpy.eye(n)), 3)
        se = numpy.sqrt(2.0 * (numpy.sum(B ** 2) - numpy.sum(numpy.diag(B) ** 2)) / s)
        exact = numpy.sum((lam + eta) ** -3.0)
        assert abs(hop.traceinv(eta, 3) - exact) < 4 * se + 1e-9 * exact


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


def test_sparse_exact_methods_vs_dense(gp):
    """The exact methods on a sparse K (the reference hands 'cholesky' to imate's
    CHOLMOD, mixed_correlation.py:250-261; its eigh of a sparse K raises,
    :76-79): the dense device copy scattered from the Morton-ordered CSR equals
    K exactly (pad included), and logdet / traceinv / eigenvalues / the
    likelihood terms match numpy on K.toarray() (<= 1e-11 relative)."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    from oracle.mixed_correlation import MixedCorrelation as OracleMC
    pts = data.generate_points(24, 2, True)          # n = 576: n_pad = 640
    D = gp.generate_correlation(pts, 0.08, 1.5, sparse=True, density=0.03,
                                device_resident=True)
    K = D.tocsr()
    n = K.shape[0]
    Kd = K.toarray()
    op = MixedCorrelation(D, imate_method='cholesky')
    assert op.sparse
    numpy.testing.assert_array_equal(op._dense().get_matrix(), Kd)
    lam = numpy.linalg.eigvalsh(Kd)
    eta = abs(lam[0]) + 0.5
    A = Kd + eta * numpy.eye(n)
    Ainv = numpy.linalg.inv(A)
    assert rel(op.logdet(eta), numpy.linalg.slogdet(A)[1]) < 1e-11
    assert rel(op.traceinv(eta, 1), numpy.trace(Ainv)) < 1e-11
    assert rel(op.traceinv(eta, 2), numpy.sum(Ainv * Ainv)) < 1e-11
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    R = numpy.column_stack([X, z])
    ld, G = op.loglik_terms([eta, eta + 1.0], X, z)
    assert _nrel(G[0], R.T @ numpy.linalg.solve(A, R)) < 1e-11
    assert rel(ld[1], numpy.linalg.slogdet(A + numpy.eye(n))[1]) < 1e-11
    ref = OracleMC(Kd, 'cholesky')
    hp = [1.0, numpy.sqrt(eta)]
    assert rel(DirectLikelihood.log_likelihood(z, X, op, False, hp),
               olk.direct_lp(z, X, ref, hp)) < 1e-10
    # 'hutchinson' logdet is Cholesky (reference :250-261)
    assert rel(MixedCorrelation(D, imate_method='hutchinson').logdet(eta),
               numpy.linalg.slogdet(A)[1]) < 1e-11
    eop = MixedCorrelation(D, imate_method='eigenvalue')
    assert numpy.max(numpy.abs(eop.eigenvalues() - lam)) < 1e-12 * numpy.max(numpy.abs(lam))
    assert rel(eop.traceinv(eta, 1), numpy.trace(Ainv)) < 1e-11
    assert rel(eop.logdet(eta), numpy.linalg.slogdet(A)[1]) < 1e-11
    with pytest.raises(numpy.linalg.LinAlgError):
        op.logdet(0.5 * abs(lam[0]))
    with pytest.raises(ValueError):
        MixedCorrelation(D, imate_method='exact').logdet(eta)


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


# ------------------------------------------------ BASELINE configs 4 and 5 ---

def _cfg_sparse(gp, name, npts, d, rho, dens):
    meta = load_json(name)
    pts = data.generate_points(npts, d, True)
    D = gp.generate_correlation(pts, rho, 1.5, sparse=True, density=dens, device_resident=True)
    return meta, pts, D


def _check_csr(D, meta):
    assert D.nnz == meta['nnz']
    K = D.tocsr()
    assert abs(K.data.sum() - meta['data_sum']) <= 1e-12 * meta['data_sum']
    assert K.data.min() == pytest.approx(meta['min_kept'], rel=1e-15)
    assert abs(K.diagonal().sum() - meta['diag_sum']) <= 1e-12 * meta['diag_sum']
    assert abs(numpy.sum(K.data ** 2) - meta['frob2']) <= 1e-12 * meta['frob2']
    rows = meta['sample_rows']
    numpy.testing.assert_array_equal(numpy.diff(K.indptr)[rows], meta['row_nnz_sample'])
    numpy.testing.assert_allclose(numpy.asarray(K.sum(axis=1)).ravel()[rows],
                                  meta['row_sums_sample'], rtol=1e-14)
    return K


def _lanczos_same_probes(sop, K, nprobe, steps, seed):
    a, b = sop.lanczos(nprobe, steps, seed)
    P = osp.rademacher_probes(K.shape[0], nprobe, seed)
    for p in range(nprobe):
        ao, bo = osp.lanczos(K, P[:, p], steps)
        k = ao.size
        assert rel(a[p, :k], ao) < 1e-9, p
        assert rel(b[p, :k - 1], bo) < 1e-9, p


def test_config4_full_size_vs_reference(gp):
    """BASELINE cfg4 at full size (N=65536, 2D, tapered Matern nu=1.5, rho=0.005,
    density 1e-3) against tests/golden/sparse_cfg4.json, made by the reference
    generator (+ the 2 argument fixes) with SuperLU exact values at three eta
    above |lambda_min|: CSR; device Lanczos vs the oracle with identical probes
    (<= 1e-9); multi-shift CG Gram vs the exact Gram (<= 1e-6 at the reference's
    rtol 1e-6, <= 1e-9 at 1e-10); SLQ logdet within 3 Monte-Carlo standard errors;
    the direct log-likelihood (SLQ logdet + CG Gram) within that error."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    from gaussian_proc import _slq
    meta, pts, D = _cfg_sparse(gp, 'sparse_cfg4.json', 256, 2, 0.005, 1e-3)
    K = _check_csr(D, meta)
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': 64, 'lanczos_degree': 30})
    _lanczos_same_probes(op.sop, K, 3, 30, 0)
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    R = numpy.column_stack([X, z])
    etas = meta['etas']
    for rtol, tol in ((1e-6, 1e-6), (1e-10, 1e-9)):
        G = op.sop.msgram(etas, R, rtol=rtol)
        for Gj, Gr in zip(G, meta['gram']):
            assert _nrel(Gj, numpy.asarray(Gr)) < tol, rtol
    q = _slq.quadrature(op.slq_nodes(), etas, _slq.FUNCS['logdet']) * op.n
    est = q.mean(axis=0)
    se = q.std(axis=0, ddof=1) / numpy.sqrt(q.shape[0])
    err = numpy.abs(est - meta['logdet'])
    assert numpy.all(err <= 3.0 * se), (err / se)
    for e, ld_se, lp_ref in zip(etas, se, meta['direct_lp']):
        lp = DirectLikelihood.log_likelihood(z, X, op, False, [1.0, numpy.sqrt(e)])
        assert abs(lp - lp_ref) <= 0.5 * 3.0 * ld_se + 1e-6 * abs(lp_ref), (e, lp, lp_ref)


def test_config4_exact_cholesky_vs_splu(gp):
    """cfg4 (N=65536) under imate_method='cholesky': the dense device copy of the
    sparse K (34 GB) and its fp64 MFMA Cholesky against the fixture's SuperLU
    logdet and exact Gram blocks (<= 1e-10) and the reference-formula lp."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    meta, pts, D = _cfg_sparse(gp, 'sparse_cfg4.json', 256, 2, 0.005, 1e-3)
    op = MixedCorrelation(D, imate_method='cholesky')
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    etas = meta['etas']
    ld, G = op.loglik_terms(etas, X, z)
    for j in range(len(etas)):
        assert rel(ld[j], meta['logdet'][j]) < 1e-10, etas[j]
        assert _nrel(G[j], numpy.asarray(meta['gram'][j])) < 1e-10, etas[j]
    e = etas[0]
    lp = DirectLikelihood.log_likelihood(z, X, op, False, [1.0, numpy.sqrt(e)])
    assert rel(lp, meta['direct_lp'][0]) < 1e-10


def test_config4_eta_below_lambda_min_raises(gp):
    """The tapered Matern is indefinite: an eta below |lambda_min|
    must raise LinAlgError (SLQ Ritz check, CG curvature check), not return."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    meta, pts, D = _cfg_sparse(gp, 'sparse_cfg4.json', 256, 2, 0.005, 1e-3)
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': 8, 'lanczos_degree': 30})
    bad = 0.5 * abs(meta['lambda_min'])
    with pytest.raises(numpy.linalg.LinAlgError):
        op.logdet(bad)
    X = data.generate_basis_functions(pts, 2)
    with pytest.raises(numpy.linalg.LinAlgError):
        op.loglik_terms([bad, 1.0], X, data.generate_data(pts, 0.2))


def test_cg_and_msgram_detect_negative_curvature(gp):
    """p^T (K + eta I) p <= 0 inside CG means K + eta I is not positive
    definite: LinAlgError (the dense path's posv behaviour), never a silent
    result. The RHS is the eigenvector of the most negative eigenvalue, so the
    first CG step meets it."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    lam, U = numpy.linalg.eigh(K.toarray())
    sop = _hip.SparseOperator.from_csr(K)
    shift = -lam[0] - 0.25                       # K + shift I has eigenvalue -0.25
    v = U[:, 0]
    with pytest.raises(numpy.linalg.LinAlgError):
        sop.cg(shift, v, rtol=1e-10)
    with pytest.raises(numpy.linalg.LinAlgError):
        sop.msgram([shift, shift + 10.0], numpy.column_stack([v, U[:, 1]]), rtol=1e-10)


def test_cg_unconverged_warns(gp):
    """scipy's cg returns an unconverged iterate silently (the reference ignores
    its info, _linear_solver.py:64,68); here it is a RuntimeWarning."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    sop = _hip.SparseOperator.from_csr(K)
    B = numpy.random.RandomState(3).randn(K.shape[0], 3)
    with pytest.warns(RuntimeWarning):
        sop.cg(3.0, B, rtol=1e-14, maxiter=2)
    with pytest.warns(RuntimeWarning):
        sop.msgram([3.0, 5.0], B, rtol=1e-14, maxiter=2)


def test_msgram_at_maxiter_applies_the_last_step(gp):
    """the multi-shift CG applies shift step k - 1 during iteration k,
    so a loop ending at maxiter with active columns must still apply its last step
    (ms_cg2_close_kernel). After k iterations each shifted solution equals plain CG
    on K + eta_j I after k steps (same Krylov space, x0 = 0): G_j = B^T x_j^(k)
    against a host CG truncated at k, for k = 1, 3, 7."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    Kd = K.toarray()
    n = Kd.shape[0]
    B = numpy.random.RandomState(11).randn(n, 3)
    etas = numpy.array([3.0, 4.5, 9.0])
    sop = _hip.SparseOperator.from_csr(K)

    def cg_steps(A, b, k):
        x = numpy.zeros_like(b)
        r = b.copy()
        p = r.copy()
        rr = r @ r
        for _ in range(k):
            Ap = A @ p
            a = rr / (p @ Ap)
            x += a * p
            r -= a * Ap
            rn = r @ r
            p = r + (rn / rr) * p
            rr = rn
        return x

    for k in (1, 3, 7):
        with pytest.warns(RuntimeWarning):
            G = sop.msgram(etas, B, rtol=1e-15, maxiter=k)
        for j, eta in enumerate(etas):
            A = Kd + eta * numpy.eye(n)
            X = numpy.column_stack([cg_steps(A, B[:, c], k) for c in range(3)])
            ref = B.T @ X
            assert numpy.max(numpy.abs(G[j] - ref)) <= 1e-10 * numpy.abs(ref).max(), (k, j)


@pytest.mark.parametrize('cols', [None, (1, 7)])
def test_msgram_compaction_bit_identical(gp, monkeypatch, cols):
    """Active-column compaction: six right-hand sides in the span of a few
    eigenvectors converge within the first poll, the seventh (random) does not;
    the block then narrows to its active columns. The Grams equal the uncompacted
    block's bit for bit (every column's arithmetic is per column), for the full
    block and a column shard, and match the exact solves."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    Kd = K.toarray()
    n = Kd.shape[0]
    lam, U = numpy.linalg.eigh(Kd)
    rng = numpy.random.RandomState(9)
    B = numpy.empty((n, 7))
    for c in range(6):
        B[:, c] = U[:, -1 - c] + 0.5 * U[:, -2 - c]
    B[:, 6] = rng.randn(n)
    etas = numpy.array([3.0, 5.0, 40.0])
    sop = _hip.SparseOperator.from_csr(K)
    monkeypatch.setenv('GPMI_MS_COMPACT', '0')
    G0 = sop.msgram(etas, B, rtol=1e-12, cols=cols)
    assert sop.msgram_compactions() == 0
    seg0 = sop.msgram_segments()
    assert len(seg0) == 1
    monkeypatch.setenv('GPMI_MS_COMPACT', '1')
    G1 = sop.msgram(etas, B, rtol=1e-12, cols=cols)
    assert sop.msgram_compactions() >= 1
    # the launch segments: the full block's width, then narrower blocks, and at
    # least the iterations to the last column's stop launched in all
    seg1 = sop.msgram_segments()
    assert len(seg1) == sop.msgram_compactions() + 1
    assert seg1[0][0] == seg0[0][0]
    assert all(seg1[q + 1][0] <= seg1[q][0] // 2 for q in range(len(seg1) - 1))
    assert sum(k for _, k in seg1) >= sop.last_cg_iterations > 0
    numpy.testing.assert_array_equal(G1, G0)
    lo, hi = cols if cols else (0, 7)
    for j, eta in enumerate(etas):
        ref = B.T @ numpy.linalg.solve(Kd + eta * numpy.eye(n), B[:, lo:hi])
        assert numpy.max(numpy.abs(G1[j] - ref)) <= 1e-9 * numpy.abs(ref).max()


def test_msgram_repeated_compactions_bit_identical(gp, monkeypatch):
    """Columns that stop in three waves (four in the span of two eigenvectors, two in
    the span of 24 spread over the spectrum, two random; ~2, ~21, ~35 iterations):
    the block narrows more than once (8 -> 4 -> 2 ...). Each compaction gathers the state of the block the previous one made (round
    6: both lived in one buffer, and the second gather overwrote what it read). The
    Grams equal the uncompacted block's bit for bit, and the exact solves."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    Kd = K.toarray()
    n = Kd.shape[0]
    lam, U = numpy.linalg.eigh(Kd)
    rng = numpy.random.RandomState(11)
    B = numpy.empty((n, 8))
    for c in range(4):
        B[:, c] = U[:, -1 - c] + 0.5 * U[:, -2 - c]
    for c in range(4, 6):   # 24 eigenvectors across the spectrum: ~21 iterations
        B[:, c] = U[:, ::24][:, :24] @ rng.randn(24)
    B[:, 6:] = rng.randn(n, 2)
    etas = numpy.array([3.0, 5.0, 40.0])
    sop = _hip.SparseOperator.from_csr(K)
    monkeypatch.setenv('GPMI_MS_COMPACT', '0')
    G0 = sop.msgram(etas, B, rtol=1e-12)
    it0 = sop.last_cg_iterations
    monkeypatch.setenv('GPMI_MS_COMPACT', '1')
    G1 = sop.msgram(etas, B, rtol=1e-12)
    assert sop.msgram_compactions() >= 2, sop.msgram_segments()
    assert sop.last_cg_iterations == it0
    numpy.testing.assert_array_equal(G1, G0)
    for j, eta in enumerate(etas):
        ref = B.T @ numpy.linalg.solve(Kd + eta * numpy.eye(n), B)
        assert numpy.max(numpy.abs(G1[j] - ref)) <= 1e-9 * numpy.abs(ref).max()


def test_msgram_compaction_then_maxiter_bit_identical(gp, monkeypatch):
    """A block that narrows (four columns stop within a few iterations) and then
    reaches maxiter with its two random columns still active: the last step lands in
    the compacted block (ms_cg2_close_kernel on it), the stopped columns' Grams come
    from the device array their compaction wrote, and everything equals the
    uncompacted block bit for bit."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    Kd = K.toarray()
    n = Kd.shape[0]
    lam, U = numpy.linalg.eigh(Kd)
    B = numpy.empty((n, 6))
    for c in range(4):
        B[:, c] = U[:, -1 - c] + 0.5 * U[:, -2 - c]
    B[:, 4:] = numpy.random.RandomState(5).randn(n, 2)
    etas = numpy.array([3.0, 6.0])
    sop = _hip.SparseOperator.from_csr(K)
    for maxiter in (17, 24):
        monkeypatch.setenv('GPMI_MS_COMPACT', '0')
        with pytest.warns(RuntimeWarning):
            G0 = sop.msgram(etas, B, rtol=1e-13, maxiter=maxiter)
        monkeypatch.setenv('GPMI_MS_COMPACT', '1')
        with pytest.warns(RuntimeWarning):
            G1 = sop.msgram(etas, B, rtol=1e-13, maxiter=maxiter)
        assert sop.msgram_compactions() >= 1, sop.msgram_segments()
        numpy.testing.assert_array_equal(G1, G0)
        for j, eta in enumerate(etas):   # the quick columns are solved
            ref = B.T @ numpy.linalg.solve(Kd + eta * numpy.eye(n), B[:, :4])
            assert numpy.max(numpy.abs(G1[j][:, :4] - ref)) <= 1e-9 * numpy.abs(ref).max()


def test_msgram_large_shifts_stay_finite(gp):
    """A large shift's zeta decays like (1 + d alpha)^-k and underflows to 0 within
    the seed system's iterations; alpha^s = alpha zeta_k / zeta_{k-1} was then 0 / 0
    (round 6: the largest eta of cfg 4's curve had a NaN Gram column). Converged
    shifts now stop (their zeta below 1e-250): every G finite and equal to the
    exact solve, while the small shifts keep their accuracy."""
    from gaussian_proc import _hip
    _, K = _small_sparse()
    Kd = K.toarray()
    n = Kd.shape[0]
    B = numpy.random.RandomState(5).randn(n, 3)
    etas = numpy.array([3.0, 30.0, 1e3, 1e6, 1e9])
    sop = _hip.SparseOperator.from_csr(K)
    G = sop.msgram(etas, B, rtol=1e-13)
    assert numpy.all(numpy.isfinite(G))
    for j, eta in enumerate(etas):
        ref = B.T @ numpy.linalg.solve(Kd + eta * numpy.eye(n), B)
        assert numpy.max(numpy.abs(G[j] - ref)) <= 1e-10 * numpy.abs(ref).max(), (eta,)


def test_config5_full_size_vs_reference(gp):
    """BASELINE cfg5 at full size (N=262144, 3D 64^3 grid, rho=0.02, density
    6e-4) against tests/golden/sparse_cfg5.json (reference generator + the 2
    argument fixes): CSR, and the device Lanczos vs the oracle with identical
    probes (<= 1e-9). Exact logdet at this size is out of reach of the host
    sparse LU (3D fill-in; test_sparse_3d_exact_logdet_vs_reference pins the same
    stencil at 32^3 against exact values); the SLQ estimate is checked for
    consistency: the 64-probe mean lies within 3 standard errors of the 20-probe
    one. The multi-shift Gram is checked against host CG (<= 1e-9), and the direct
    lp against the oracle's formula on a host operator with the same probes."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc import _slq
    meta, pts, D = _cfg_sparse(gp, 'sparse_cfg5.json', 64, 3, 0.02, 6e-4)
    K = _check_csr(D, meta)
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': 64, 'lanczos_degree': 30})
    _lanczos_same_probes(op.sop, K, 2, 30, 0)
    eta = 1.1 * abs(meta['lambda_min']) + 0.1
    q = _slq.quadrature(op.slq_nodes(), [eta], _slq.FUNCS['logdet'])[:, 0] * op.n
    se = q.std(ddof=1) / numpy.sqrt(q.size)
    assert abs(q[:20].mean() - q.mean()) <= 3.0 * se * numpy.sqrt(64 / 20.0)
    # beyond the CSR: the multi-shift CG Gram at two eta above |lambda_min| against
    # host CG (the oracle's solve, rtol 1e-12, thread pool over the columns), and
    # the direct lp (_direct_likelihood.py:31-83) on the device operator (8-probe
    # SLQ logdet + CG Gram) against the oracle formula on the host operator with
    # the same 8 probes (oracle.sparse.slq) and the host CG solves
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    R = numpy.column_stack([X, z])
    etas = [eta, eta + 1.0]
    G = op.sop.msgram(etas, R, rtol=1e-10)
    host = _HostSparseOperator(K, 8, 30, 0)
    for e, Gj in zip(etas, G):
        assert _nrel(Gj, R.T @ host.solve(e, R)) < 1e-9, e
    op8 = MixedCorrelation(D, imate_method='slq',
                           imate_options={'num_samples': 8, 'lanczos_degree': 30})
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    from oracle import likelihood as olk
    assert rel(op8.logdet(eta), host.logdet(eta)) < 1e-9
    for hp in ([1.0, numpy.sqrt(eta)], [0.5, 0.5 * numpy.sqrt(eta + 1.0)]):
        lp_ref = olk.direct_lp(z, X, host, hp)
        # the operator's CG at the reference's rtol 1e-6 (_linear_solver.py:24): within
        # the north star's lp bound; at rtol 1e-10 the same formula to 1e-9
        op8.cg_rtol = 1e-6
        lp = DirectLikelihood.log_likelihood(z, X, op8, False, hp)
        assert rel(lp, lp_ref) < 1e-6, hp
        op8.cg_rtol = 1e-10
        lp = DirectLikelihood.log_likelihood(z, X, op8, False, hp)
        assert rel(lp, lp_ref) < 1e-9, hp


class _HostSparseOperator(object):
    """Host operator for the oracle's likelihood formulas on a sparse K: SLQ
    logdet with the device's counter-based probes (oracle.sparse.slq) and solves
    by scipy CG at rtol 1e-12, probes and columns on a thread pool."""

    def __init__(self, K, nprobe, steps, seed):
        self.K = K.tocsr()
        self.n = K.shape[0]
        self.P = osp.rademacher_probes(self.n, nprobe, seed)
        self.steps = steps
        self._nodes = None

    def logdet(self, eta):
        from concurrent.futures import ThreadPoolExecutor
        if self._nodes is None:
            with ThreadPoolExecutor(16) as ex:
                ab = list(ex.map(lambda p: osp.lanczos(self.K, self.P[:, p], self.steps),
                                 range(self.P.shape[1])))
            self._nodes = [osp.slq_nodes(a, b) for a, b in ab]
        return self.n * numpy.mean([numpy.sum(w * numpy.log(t + eta)) for t, w in self._nodes])

    def solve(self, eta, Y):
        import scipy.sparse
        import scipy.sparse.linalg
        from concurrent.futures import ThreadPoolExecutor
        A = (self.K + eta * scipy.sparse.identity(self.n, format='csr')).tocsr()
        Y2 = numpy.asarray(Y, dtype=float)
        cols = Y2[:, None] if Y2.ndim == 1 else Y2

        def one(c):
            x, info = scipy.sparse.linalg.cg(A, cols[:, c], rtol=1e-12, atol=0.0,
                                             maxiter=20 * self.n)
            assert info == 0
            return x
        with ThreadPoolExecutor(16) as ex:
            out = numpy.column_stack(list(ex.map(one, range(cols.shape[1]))))
        return out[:, 0] if Y2.ndim == 1 else out


def test_sparse_3d_exact_logdet_vs_reference(gp):
    """cfg5's 3-D stencil on a 32^3 grid (N=32768, rho and density scaled so a row
    keeps cfg5's neighbours) against tests/golden/sparse_3d32.json, made by the
    reference generator (+ the 2 argument fixes) with SuperLU exact values at
    three eta above |lambda_min|: CSR; multi-shift CG Gram <= 1e-9 at rtol 1e-10
    (<= 1e-6 at the reference's rtol 1e-6); the 64-probe SLQ logdet within 3
    Monte-Carlo standard errors of the exact logdet; the direct lp within that
    error of the reference's lp on the exact operator."""
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    from gaussian_proc import _slq
    meta, pts, D = _cfg_sparse(gp, 'sparse_3d32.json', 32, 3, 0.04, 4.8e-3)
    K = _check_csr(D, meta)
    op = MixedCorrelation(D, imate_method='slq',
                          imate_options={'num_samples': 64, 'lanczos_degree': 30})
    _lanczos_same_probes(op.sop, K, 3, 30, 0)
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    R = numpy.column_stack([X, z])
    etas = meta['etas']
    for rtol, tol in ((1e-6, 1e-6), (1e-10, 1e-9)):
        G = op.sop.msgram(etas, R, rtol=rtol)
        for Gj, Gr in zip(G, meta['gram']):
            assert _nrel(Gj, numpy.asarray(Gr)) < tol, rtol
    q = _slq.quadrature(op.slq_nodes(), etas, _slq.FUNCS['logdet']) * op.n
    est = q.mean(axis=0)
    se = q.std(axis=0, ddof=1) / numpy.sqrt(q.shape[0])
    err = numpy.abs(est - meta['logdet'])
    assert numpy.all(err <= 3.0 * se), (err / se)
    for e, ld_se, lp_ref in zip(etas, se, meta['direct_lp']):
        lp = DirectLikelihood.log_likelihood(z, X, op, False, [1.0, numpy.sqrt(e)])
        assert abs(lp - lp_ref) <= 0.5 * 3.0 * ld_se + 1e-6 * abs(lp_ref), (e, lp, lp_ref)


@pytest.mark.parametrize('world', [2, 4, 8])
def test_rank_shards_equal_one_device(gp, world):
    """The bench's sparse shards at N ranks, run one after another on one device:
    every rank's probe block of the Lanczos (counter-based probes at its offset,
    imate's plain recurrence and DCGS2) and right-hand-side column block of the
    multi-shift CG (gpmi_sp_msgram_cols; 1-3 columns at N = 8) together equal the
    single-device results to 1e-9 (other block widths take other SpMM kernels)."""
    from gaussian_proc import _hip
    from gaussian_proc.sweep import shard
    _, K = _small_sparse()
    n = K.shape[0]
    sop = _hip.SparseOperator.from_csr(K)
    nprobe, steps, seed = 20, 12, 3
    for orth in (0, -1):
        a, b = sop.lanczos(nprobe, steps, seed, orthogonalize=orth)
        for r in range(world):
            lo, hi, _ = shard(nprobe, world, r)
            if hi > lo:
                ar, br = sop.lanczos(hi - lo, steps, seed, probe_offset=lo, orthogonalize=orth)
                # (other block widths run other SpMM kernels: rounding-level differences)
                assert rel(ar, a[lo:hi]) < 1e-9 and rel(br, b[lo:hi]) < 1e-9, (world, r, orth)
    rng = numpy.random.RandomState(world)
    B = rng.randn(n, 7)
    etas = numpy.array([2.5, 4.0, 10.0])
    G = sop.msgram(etas, B, rtol=1e-10)
    for r in range(world):
        lo, hi, _ = shard(7, world, r)
        if hi > lo:
            Gc = sop.msgram(etas, B, rtol=1e-10, cols=(lo, hi))
            assert _nrel(Gc, G[:, :, lo:hi]) < 1e-9, (world, r)
