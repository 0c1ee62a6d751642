"""eta-grid sharding + one all-gather (gaussian_proc.sweep) on CPU with the
gloo backend, world size 2 (the multi-GPU path uses the same code over RCCL).
The device operator is replaced by an exact numpy stand-in with the same
``loglik_terms`` contract, so this runs without a GPU."""

import os
import socket

import numpy
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from gaussian_proc.sweep import shard, eta_sweep
from gaussian_proc._likelihood._direct_likelihood import _lp_from_terms


class _NumpyOperator(object):
    def __init__(self, K):
        self.K = K

    def loglik_terms(self, etas, X, z):
        R = numpy.column_stack([X, z])
        lds, gs = [], []
        for e in etas:
            A = self.K + e * numpy.eye(self.K.shape[0])
            L = numpy.linalg.cholesky(A)
            W = numpy.linalg.solve(L, R)
            lds.append(2.0 * numpy.sum(numpy.log(numpy.diag(L))))
            gs.append(W.T @ W)
        return numpy.array(lds), numpy.array(gs)


def _problem():
    rng = numpy.random.RandomState(0)
    n = 60
    pts = rng.rand(n, 2)
    d = numpy.sqrt(((pts[:, None, :] - pts[None, :, :]) ** 2).sum(-1)) / 0.3
    K = (1 + numpy.sqrt(3) * d) * numpy.exp(-numpy.sqrt(3) * d)
    X = numpy.column_stack([numpy.ones(n), pts])
    z = numpy.sin(3 * pts[:, 0]) + 0.1 * rng.randn(n)
    return K, X, z


def _worker(rank, world, port, etas, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    K, X, z = _problem()
    ld, lp = eta_sweep(_NumpyOperator(K), X, z, etas, sigma=1.0)
    out_q.put((rank, ld, lp))
    dist.barrier()
    dist.destroy_process_group()


class _FakeSparse(object):
    """Exact numpy Lanczos with the counter-based probes (stand-in for the
    device SparseOperator.lanczos in a CPU-only process)."""

    def __init__(self, K, steps):
        self.K = K
        self.steps = steps

    def lanczos(self, nprobe, steps, seed=0, probe_offset=0, orthogonalize=-1):
        from oracle import sparse as osp
        P = osp.rademacher_probes(self.K.shape[0], probe_offset + nprobe, seed)[:, probe_offset:]
        a = numpy.zeros((nprobe, steps))
        b = numpy.zeros((nprobe, steps))
        for p in range(nprobe):
            ao, bo = osp.lanczos(self.K, P[:, p], steps, reorth=orthogonalize != 0)
            a[p, :ao.size] = ao
            b[p, :bo.size] = bo
        return a, b


class _SparseMixed(object):
    def __init__(self, K):
        self.sop = _FakeSparse(K, 12)
        self.num_samples = 5
        self.lanczos_degree = 12
        self.seed = 3
        self.n = K.shape[0]


def _slq_worker(rank, world, port, etas, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from gaussian_proc.sweep import slq_sweep
    K, _, _ = _problem()
    res = slq_sweep(_SparseMixed(K + 0.5 * numpy.eye(K.shape[0])), etas)
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_slq_sweep_probe_sharding_gloo():
    from gaussian_proc.sweep import slq_sweep
    etas = numpy.array([0.5, 1.0, 4.0])
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slq_worker, args=(r, 2, port, etas, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    K, _, _ = _problem()
    ref = slq_sweep(_SparseMixed(K + 0.5 * numpy.eye(K.shape[0])), etas, group=False)
    for _, r in res:
        for k in ('logdet', 'traceinv', 'traceinv2'):
            numpy.testing.assert_allclose(r[k], ref[k], rtol=1e-12)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_covers_grid_exactly_once():
    for num in (1, 7, 64, 65):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi, per = shard(num, world, r)
                assert hi - lo <= per
                seen.extend(range(lo, hi))
            assert seen == list(range(num))


@pytest.mark.parametrize('world,neta', [(2, 9), (2, 8)])
def test_eta_sweep_gloo_matches_single_process(world, neta):
    etas = numpy.logspace(-2, 2, neta)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, etas, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    K, X, z = _problem()
    ld_ref, lp_ref = eta_sweep(_NumpyOperator(K), X, z, etas, sigma=1.0, group=False)
    n, m = X.shape
    for _, ld, lp in res:
        numpy.testing.assert_allclose(ld, ld_ref, rtol=1e-13)
        numpy.testing.assert_allclose(lp, lp_ref, rtol=1e-13)
    # the stand-in's lp is the reference formula
    from oracle.mixed_correlation import MixedCorrelation
    from oracle import likelihood as olk
    ref = MixedCorrelation(K, 'cholesky')
    for e, v in zip(etas, lp_ref):
        assert abs(v - olk.direct_lp(z, X, ref, [1.0, numpy.sqrt(e)])) <= 1e-10 * abs(v)


def _slq_bad_worker(rank, world, port, etas, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from gaussian_proc.sweep import slq_sweep
    K, _, _ = _problem()
    try:
        slq_sweep(_SparseMixed(K - 2.0 * numpy.eye(K.shape[0])), etas)
        out_q.put((rank, 'returned'))
    except numpy.linalg.LinAlgError:
        out_q.put((rank, 'LinAlgError'))
    dist.barrier()
    dist.destroy_process_group()


def test_slq_sweep_rejects_eta_below_lambda_min_on_every_rank():
    """K - 2I is indefinite (lambda_min(K) < 2): an eta grid reaching below
    |lambda_min| must raise LinAlgError on every rank alike (the check runs after
    the all-gather, so no rank is left waiting in a collective)."""
    etas = numpy.array([0.5, 1.0, 4.0])
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slq_bad_worker, args=(r, 2, port, etas, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r for _, r in res) == ['LinAlgError', 'LinAlgError']


def test_slq_quadrature_shift_check():
    from gaussian_proc import _slq
    nodes = [(numpy.array([-1.5, 0.2, 3.0]), numpy.array([0.2, 0.3, 0.5]))]
    with pytest.raises(numpy.linalg.LinAlgError):
        _slq.quadrature(nodes, [1.0, 2.0], _slq.FUNCS['logdet'])
    q = _slq.quadrature(nodes, [1.6, 2.0], _slq.FUNCS['logdet'])
    assert numpy.all(numpy.isfinite(q))


def _bench_worker(rank, world, port, out_q):
    """bench.py's strong-scaled step plumbing on gloo: the rank's eta block of
    the 64-point cfg3 curve and the one all-gather of the [eta, logdet, lp] rows
    (the numbers here stand in for the device's)."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import sys
    import types
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    args = types.SimpleNamespace(scaling='strong', eta_total=64, eta_per_rank=64)
    etas, own, per, gsize = bench.eta_block(args, world, rank)
    rows = numpy.stack([etas, numpy.log(etas), -etas], axis=1)
    allrows = bench.gather_rows(rows, world, dist, torch)
    out_q.put((rank, own, per, gsize, allrows))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_bench_strong_scaling_blocks_and_all_gather_gloo(world):
    """The 64-point curve split over N ranks (contiguous blocks, last block
    padded by repeating its eta), gathered once: every rank ends with the whole
    curve in order."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    grid = numpy.logspace(-3, 3, 64)
    owns = [r[1] for r in res]
    assert sum(owns) == 64
    for rank, own, per, gsize, allrows in res:
        assert gsize == 64 and allrows.shape == (world * per, 3)
        got = numpy.concatenate([allrows[r * per:r * per + owns[r], 0] for r in range(world)])
        numpy.testing.assert_array_equal(got, grid)


class _Der1Operator(object):
    """Stand-in whose batched der1 raises LinAlgError for eta < 1e-3 (as a
    device operator raises for K + eta I not positive definite)."""
    imate_method = 'cholesky'


def _der1_worker(rank, world, port, log_etas, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from gaussian_proc import sweep
    from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood

    def fake(z, X, K_mixed, les):
        les = numpy.asarray(les, dtype=float)
        if numpy.any(les < -3.0):
            raise numpy.linalg.LinAlgError('not positive definite')
        return numpy.tanh(les - 0.7)
    ProfileLikelihood.log_likelihood_der1_eta_batch = staticmethod(fake)
    outs = []
    for le in log_etas:
        try:
            outs.append(sweep.der1_sweep(_Der1Operator(), None, None, le, group=None))
        except numpy.linalg.LinAlgError:
            outs.append('LinAlgError')
    # the default is local (group=False): no collective, runs on one rank alone
    outs.append(sweep.der1_sweep(_Der1Operator(), None, None, [0.0, 1.0]))
    out_q.put((rank, outs))
    dist.barrier()
    dist.destroy_process_group()


def test_der1_sweep_error_raises_on_every_rank_gloo():
    """A LinAlgError in one rank's shard raises on every rank after the
    all-gather (no rank is left blocked in it); a clean batch is gathered in
    order; without an explicit group der1_sweep stays local."""
    good = numpy.linspace(-1.0, 2.0, 5)
    bad = numpy.array([0.0, 0.5, 1.0, -4.0])       # the last eta lands on rank 1
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_der1_worker, args=(r, 2, port, [good, bad], q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, outs in res:
        numpy.testing.assert_array_equal(outs[0], numpy.tanh(good - 0.7))
        assert outs[1] == 'LinAlgError'
        numpy.testing.assert_array_equal(outs[2], numpy.tanh(numpy.array([0.0, 1.0]) - 0.7))


class _FakeSparseGram(_FakeSparse):
    rhs_cols = 0

    def set_rhs(self, B):   # the resident block (gpmi_sp_set_rhs) stand-in
        self._rhs = numpy.array(B, dtype=float)
        self.rhs_cols = self._rhs.shape[1]

    def msgram(self, etas, R, rtol=1e-6, maxiter=None, cols=None):
        if R is None:
            R = self._rhs
        n = self.K.shape[0]
        G = numpy.array([R.T @ numpy.linalg.solve(self.K + e * numpy.eye(n), R)
                         for e in etas])
        return G if cols is None else G[:, :, cols[0]:cols[1]]


class _SparseMixedGram(_SparseMixed):
    def __init__(self, K):
        _SparseMixed.__init__(self, K)
        self.sop = _FakeSparseGram(K, 12)


def _slq_gram_worker(rank, world, port, etas, out_q, resident=False):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from gaussian_proc.sweep import slq_gram_sweep
    K, X, z = _problem()
    R = numpy.column_stack([X, z])
    op = _SparseMixedGram(K + 0.5 * numpy.eye(K.shape[0]))
    if resident:
        op.sop.set_rhs(R)   # the bench's form: [X z] resident, the sweep given R = None
        R = None
    out_q.put((rank, slq_gram_sweep(op, etas, R)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('resident', [False, True])
def test_slq_gram_sweep_gloo(resident):
    """slq_gram_sweep: the probe-sharded SLQ curves (all-gathered, equal on every
    rank) and the multi-shift Gram blocks computed together (second host thread),
    the Gram split by right-hand-side columns over the ranks and all-gathered after
    the Lanczos; each rank's eta block of the result, whose union is the
    single-process result. ``resident``: the right-hand sides made resident first
    (sop.set_rhs) and the sweep given R = None, as the bench runs it."""
    from gaussian_proc.sweep import slq_gram_sweep
    etas = numpy.array([0.5, 1.0, 2.0, 4.0, 8.0])
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slq_gram_worker, args=(r, 2, port, etas, q, resident))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    K, X, z = _problem()
    R = numpy.column_stack([X, z])
    op = _SparseMixedGram(K + 0.5 * numpy.eye(K.shape[0]))
    curves, (lo, hi), G = slq_gram_sweep(op, etas, R, group=False)
    assert (lo, hi) == (0, etas.size)
    blocks = []
    for _, (c, (l, h), g) in res:
        for k in ('logdet', 'traceinv', 'traceinv2'):
            numpy.testing.assert_allclose(c[k], curves[k], rtol=1e-12)
        blocks.append(g)
    numpy.testing.assert_allclose(numpy.concatenate(blocks), G, rtol=1e-12)


class _FakeSparseGramCurv(_FakeSparseGram):
    """msgram that meets negative curvature on the last right-hand-side column
    (the device check depends on the columns a rank solves)."""

    def msgram(self, etas, R, rtol=1e-6, maxiter=None, cols=None):
        c_hi = R.shape[1] if cols is None else cols[1]
        if c_hi == R.shape[1]:
            raise numpy.linalg.LinAlgError('negative curvature p^T (K + eta I) p <= 0')
        return _FakeSparseGram.msgram(self, etas, R, rtol, maxiter, cols)


def _slq_gram_curv_worker(rank, world, port, etas, split, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from gaussian_proc.sweep import slq_gram_sweep
    K, X, z = _problem()
    R = numpy.column_stack([X, z])
    op = _SparseMixed(K + 0.5 * numpy.eye(K.shape[0]))
    op.sop = _FakeSparseGramCurv(op.sop.K, 12)
    outs = []
    try:
        slq_gram_sweep(op, etas, R, split=split)
        outs.append('ok')
    except numpy.linalg.LinAlgError:
        outs.append('LinAlgError')
    # the group is still usable afterwards: a clean all-gather in step
    from gaussian_proc.sweep import _all_gather_rows
    outs.append(_all_gather_rows(dist, None, numpy.array([[float(rank)]]), world).ravel().tolist())
    out_q.put((rank, outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('split', ['columns', 'eta'])
def test_slq_gram_sweep_curvature_on_one_rank_raises_everywhere_gloo(split):
    """Negative curvature in ONE rank's multi-shift CG (its column shard holds the
    offending right-hand side, or only its eta block runs the full CG): every rank
    raises LinAlgError after the collectives, none is left blocked in one."""
    etas = numpy.array([0.5, 1.0, 2.0, 4.0])
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slq_gram_curv_worker, args=(r, 2, port, etas, split, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, outs in res:
        assert outs[0] == 'LinAlgError'
        assert outs[1] == [0.0, 1.0]
