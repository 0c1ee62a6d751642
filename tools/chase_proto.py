"""Dev prototype (numpy) of the band -> tridiagonal bulge chase the device
implements (gpmi_chase.hip), with its exact task decomposition, lower-triangle
storage and wavefront schedule, checked against numpy's eigenvalues.

Sweep s annihilates column s below the subdiagonal; its task k works on the row
block J_k = [s + 1 + k b, s + 1 + (k + 1) b):
  k = 0: reflector H from A[J_0, s];  k >= 1: from the first column c = s + 1 +
  (k - 1) b of the bulge block F = A[J_k, J_{k-1}]
  F <- H F (k >= 1; column c becomes (beta, 0 ...)), D = A[J_k, J_k] <- H D H,
  E = A[J_{k+1}, J_k] <- E H (creates the next bulge).
Task (s, k) may run once (s - 1, k + 2) is done: wavefront t = 3 s + k; tasks of
one wavefront touch disjoint rows.
"""
import sys

import numpy


def house(x):
    """LAPACK dlarfg: H x = beta e1, H = I - tau v v^T, v[0] = 1."""
    x0 = x[0]
    nb2 = float(numpy.dot(x[1:], x[1:]))
    v = numpy.zeros_like(x)
    v[0] = 1.0
    if nb2 == 0.0:
        return v, 0.0, x0
    nrm = numpy.sqrt(x0 * x0 + nb2)
    beta = -nrm if x0 >= 0 else nrm
    tau = (beta - x0) / beta
    v[1:] = x[1:] / (x0 - beta)
    return v, tau, beta


def task(A, n, b, s, k):
    """One chase task on the lower triangle of A (upper never read)."""
    r0 = s + 1 + k * b
    if r0 >= n:
        return False
    r1 = min(r0 + b, n)
    if k == 0:
        col = s
    else:
        col = s + 1 + (k - 1) * b
    x = A[r0:r1, col].copy()
    v, tau, beta = house(x)
    if k == 0:
        A[r0, s] = beta
        A[r0 + 1:r1, s] = 0.0
    else:
        c0, c1 = col, col + b
        F = A[r0:r1, c0:c1]
        wF = F.T @ v
        F -= tau * numpy.outer(v, wF)
        F[:, 0] = 0.0
        F[0, 0] = beta
    if tau != 0.0:
        L = numpy.tril(A[r0:r1, r0:r1])
        D = L + numpy.tril(L, -1).T
        p = tau * (D @ v)
        w = p - 0.5 * tau * (v @ p) * v
        D -= numpy.outer(v, w) + numpy.outer(w, v)
        A[r0:r1, r0:r1] = numpy.tril(D) + numpy.triu(A[r0:r1, r0:r1], 1)
        e0, e1 = r1, min(r1 + b, n)
        if e1 > e0:
            E = A[e0:e1, r0:r1]
            q = E @ v
            E -= tau * numpy.outer(q, v)
    return True


def chase(B, b):
    n = B.shape[0]
    A = numpy.tril(B).copy()
    kmax = (n + b - 1) // b + 1
    t = 0
    while True:
        did = False
        for s in range(0, min(t // 3, n - 2) + 1):
            k = t - 3 * s
            if 0 <= k <= kmax and s <= n - 3:
                did |= task(A, n, b, s, k)
        if not did and t // 3 > n - 2:
            break
        t += 1
    d = numpy.diag(A).copy()
    e = numpy.diag(A, -1).copy()
    # everything below the subdiagonal must be zero
    assert numpy.max(numpy.abs(numpy.tril(A, -2))) < 1e-12 * numpy.max(numpy.abs(d)), \
        numpy.max(numpy.abs(numpy.tril(A, -2)))
    return d, e, t


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rng = numpy.random.RandomState(0)
    M = rng.randn(n, n)
    M = M + M.T
    i, j = numpy.indices((n, n))
    B = numpy.where(numpy.abs(i - j) <= b, M, 0.0)
    d, e, T = chase(B, b)
    Tm = numpy.diag(d) + numpy.diag(e, 1) + numpy.diag(e, -1)
    lam = numpy.linalg.eigvalsh(Tm)
    ref = numpy.linalg.eigvalsh(B)
    print('n %d b %d wavefronts %d  max eig err %.2e' % (n, b, T, numpy.max(numpy.abs(lam - ref))))


if __name__ == '__main__':
    main()
