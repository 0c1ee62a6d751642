"""Host-side pieces of bench.py (CPU): the thread-pool sparse CPU baseline
reproduces the oracle's SLQ logdet with the device's probes, and the sparse
step byte model counts what its docstring says."""

import os
import sys

import numpy
import scipy.sparse
import scipy.sparse.linalg

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
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
    ref = osp.slq(K, etas, P, 12)['logdet']
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
    b = bench.sparse_step_bytes(n, nnz, 4, 3, 2, 10)
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
