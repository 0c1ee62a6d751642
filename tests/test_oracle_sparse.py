"""Pin the sparse (tapered) oracle and the SLQ restatement — CPU only."""
import numpy
import pytest
import scipy.sparse.linalg

from oracle import data, sparse
from _util import load_json, load_npz


@pytest.mark.parametrize('case', [0, 1, 2])
def test_sparse_assembly_matches_reference(case):
    meta = load_json('sparse.json')[case]
    arr = load_npz('sparse_small.npz')
    pts = data.generate_points(meta['num_points'], meta['dimension'], True)
    K, tau = sparse.sparse_correlation(pts, meta['correlation_scale'], meta['nu'],
                                       meta['density'])
    name = meta['name']
    numpy.testing.assert_array_equal(K.indptr, arr[name + '_indptr'])
    numpy.testing.assert_array_equal(K.indices, arr[name + '_indices'])
    numpy.testing.assert_allclose(K.data, arr[name + '_data'], rtol=0, atol=4e-16)
    assert K.nnz == meta['nnz']
    assert tau < meta['min_kept']


def test_threshold_raises_below_unit_adjacency():
    with pytest.raises(ValueError):
        sparse.kernel_threshold(100, 2, 0.001, numpy.array([0.1, 0.1]), 1.5)


def test_slq_matches_exact_within_mc_error():
    pts = data.generate_points(20, 2, True)
    K, _ = sparse.sparse_correlation(pts, 0.1, 1.5, 0.05)
    n = K.shape[0]
    etas = [2.0, 5.0]   # the tapered matrix is indefinite (lambda_min ~ -1.47)
    probes = sparse.rademacher_probes(n, 64, seed=7)
    est = sparse.slq(K, etas, probes, steps=30)
    Kd = K.toarray()
    for e, ld in zip(etas, est['logdet']):
        exact = numpy.linalg.slogdet(Kd + e * numpy.eye(n))[1]
        assert abs(ld - exact) < 0.02 * abs(exact) + 2.0
    for e, ti in zip(etas, est['traceinv']):
        exact = numpy.trace(numpy.linalg.inv(Kd + e * numpy.eye(n)))
        assert abs(ti - exact) < 0.03 * exact


def test_rademacher_probes_are_pm1_and_deterministic():
    p1 = sparse.rademacher_probes(1000, 4, seed=3)
    p2 = sparse.rademacher_probes(1000, 4, seed=3)
    numpy.testing.assert_array_equal(p1, p2)
    assert set(numpy.unique(p1)) == {-1.0, 1.0}
    assert abs(p1.mean()) < 0.1
