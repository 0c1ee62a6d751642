"""Dev check: 'slq' over the resident dense K at N = grid^2 against the oracle:
dense_mm rows vs numpy, the device Lanczos vs the oracle Lanczos (same probes,
host matvecs), and both SLQ logdets vs the exact one (device Cholesky).
usage: dense_slq_check.py [grid] [nprobe]"""
import os
import sys
import time

import numpy

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'gaussian-process-param-estimation_amd')]
from gaussian_proc import generate_correlation, _data, _slq, _hip  # noqa: E402
from gaussian_proc._mixed_correlation import MixedCorrelation  # noqa: E402
from oracle import sparse as osp  # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 128
nprobe = int(sys.argv[2]) if len(sys.argv) > 2 else 4
pts = _data.generate_points(grid, 2, True)
D = generate_correlation(pts, 0.1, 1.5, device_resident=True)
K = D.op.get_matrix()
n = K.shape[0]
sop = _hip.SparseOperator.from_dense(D.op)
rng = numpy.random.RandomState(0)
X = rng.randn(n, 20)
Y = sop.spmm(0.0, X)
rows = rng.choice(n, 64, replace=False)
print('n=%d dense_mm rows rel err %.2e' % (n, numpy.max(numpy.abs(Y[rows] - K[rows] @ X))
                                          / numpy.max(numpy.abs(K[rows] @ X))), flush=True)
steps = 30
a, b = sop.lanczos(nprobe, steps, 0)
P = osp.rademacher_probes(n, nprobe, 0)
etas = numpy.array([1e-3, 1.0, 1e3])
t0 = time.perf_counter()
for p in range(nprobe):
    ao, bo = osp.lanczos(K, P[:, p], steps)
    k = ao.size
    print('probe %d: alpha rel %.2e beta rel %.2e (k=%d)' % (
        p, numpy.max(numpy.abs(a[p, :k] - ao) / numpy.abs(ao)),
        numpy.max(numpy.abs(b[p, :k - 1] - bo) / numpy.abs(bo)), k), flush=True)
ref = osp.slq(K, etas, P, steps)
print('oracle slq %.1f s' % (time.perf_counter() - t0))
nodes = _slq.nodes(a, b)
est = n * _slq.quadrature(nodes, etas, numpy.log).mean(axis=0)
ex = MixedCorrelation(D, imate_method='cholesky')
for i, e in enumerate(etas):
    print('eta %g: exact %.6e device slq %.6e oracle slq %.6e' % (e, ex.logdet(e), est[i],
                                                                   ref['logdet'][i]))
