"""Host-side pieces of bench.py (CPU): the thread-pool sparse CPU baseline
reproduces the oracle's SLQ logdet with the device's probes, the sparse step
byte model counts what its docstring says, and ``--gpus N`` starts and checks
N ranks."""

import os
import sys

import numpy
import pytest
import scipy.sparse
import scipy.sparse.linalg

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'bench.py')
from oracle import sparse as osp  # noqa: E402


def _spd(n, seed=0):
    rng = numpy.random.RandomState(seed)
    r = numpy.repeat(numpy.arange(n), 6)
    c = (r + rng.randint(-20, 21, r.size)) % n
    A = scipy.sparse.csr_matrix((rng.rand(r.size) * 0.1, (r, c)), shape=(n, n))
    return (A + A.T + scipy.sparse.identity(n)).tocsr()


def test_cpu_baseline_sparse_thread_pool():
    n = 3000
    K = _spd(n)
    rng = numpy.random.RandomState(1)
    X = numpy.column_stack([numpy.ones(n), rng.rand(n)])
    z = rng.randn(n)
    etas = numpy.array([0.1, 0.5, 1.0, 2.0])
    cb = bench.cpu_baseline_sparse(K, X, z, etas, 4, 12, 5, 0.2, workers=3)
    assert cb['value'] > 0 and cb['cores'] == 3 and cb['threads'] == 3
    P = osp.rademacher_probes(n, 4, 5)
    ref = osp.slq(K, etas, P, 12, reorth=False)['logdet']
    numpy.testing.assert_allclose(cb['logdet'], ref, rtol=1e-12)
    # the solved Gram columns R^T (K + eta I)^-1 r_c (rtol 1e-6) against a direct solve
    R = numpy.column_stack([X, z])
    assert cb['gram_columns']
    for j, c, g in cb['gram_columns']:
        ex = R.T @ scipy.sparse.linalg.spsolve((K + etas[j] * scipy.sparse.identity(n)).tocsc(),
                                               R[:, c])
        assert numpy.max(numpy.abs(g - ex)) <= 1e-5 * numpy.max(numpy.abs(ex))


def test_sparse_step_bytes_model():
    n, nnz = 1000, 20000
    p = bench.sparse_step_bytes(n, nnz, 4, 3, 2, 10)     # imate's default orthogonalize = 0
    csr = 12.0 * nnz + 8.0 * (n + 1)
    assert p['lanczos'] == 3 * (csr + 6 * 8.0 * n * 4) and p['lanczos_basis_reads'] == 0.0
    assert p['cg'] == 10 * (csr + 9 * 8.0 * n * 2)
    b = bench.sparse_step_bytes(n, nnz, 4, 3, 2, 10, orthogonalize=-1)
    csr = 12.0 * nnz + 8.0 * (n + 1)
    bl, bc = 8.0 * n * 4, 8.0 * n * 2
    lz = 0.0
    for k in range(3):
        lz += csr + 2 * bl + (k + 2) * bl + (k + 4) * bl
    lz += 4 * bl
    assert b['lanczos'] == lz
    assert b['lanczos_basis_reads'] == sum(2 * k * bl for k in range(3)) + 3 * bl
    assert b['cg'] == 10 * (csr + 9 * bc)
    assert b['total'] == b['lanczos'] + b['cg']
    # the compacted CG: each launch segment at its own width
    c = bench.sparse_step_bytes(n, nnz, 4, 3, 12, 90, cg_segments=[(12, 42), (1, 49)])
    assert c['cg'] == 42 * (csr + 9 * 8.0 * n * 12) + 49 * (csr + 9 * 8.0 * n * 1)
    assert c['lanczos'] == p['lanczos']


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith('{')]
    assert lines, out
    import json
    return json.loads(lines[-1])


@pytest.mark.parametrize('world', [2, 3])
def test_bench_gpus_n_launches_n_ranks(world):
    """`python bench.py --gpus N` (no torch.distributed environment) starts N
    ranks itself (launch_ranks: torch.distributed.run as a child process), every
    rank checks the world size against --gpus, and the gathered eta blocks cover
    the 64-point curve once, in order (--launch-check: no device, gloo)."""
    import subprocess
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    out = subprocess.run([sys.executable, BENCH, '--gpus', str(world), '--launch-check'],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    d = _json_line(out.stdout)
    assert d['n_gpus'] == world and d['gpus_arg'] == world
    assert d['ranks'] == list(range(world))
    numpy.testing.assert_array_equal(d['curve_etas'], numpy.logspace(-3, 3, 64))


def test_bench_rejects_world_size_other_than_gpus():
    """A job whose world size is not --gpus fails loudly instead of reporting
    the wrong n_gpus."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    out = subprocess.run([sys.executable, BENCH, '--gpus', '2', '--launch-check'],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert '--gpus 2 but the job has 1 ranks' in out.stderr
