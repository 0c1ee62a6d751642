"""numpy prototype of the block cyclic reduction (odd-even elimination) banded
solve of B + eta I (dev tool; the device form is csrc/gpmi_bcr.hip): B is block
tridiagonal with b x b blocks, D_i = B_ii + eta I, F_i = B_{i+1,i}. Per level
the odd blocks are eliminated independently (Cholesky L_i of D_i, W_l = L_i^-1
F_{i-1}, W_r = L_i^-1 F_i^T, Z_i = L_i^-1 Y_i), then every even block j gets
  D_j' = D_j - W_r(j-1)^T W_r(j-1) - W_l(j+1)^T W_l(j+1)
  Y_j' = Y_j - W_r(j-1)^T Z_{j-1} - W_l(j+1)^T Z_{j+1}
  F_{j/2}' = -W_r(j+1)^T W_l(j+1)
(the Schur complement on the even blocks; it is a block Cholesky of the
odd-even permuted matrix). logdet = sum of 2 log diag(L_i) over every
eliminated block, Y^T (B + eta I)^-1 Y = sum of Z_i^T Z_i."""
import numpy
import scipy.linalg


def bcr(Dl, Fl, Yl):
    """Dl: list of b x b SPD blocks, Fl: list of couplings F_i = A[i+1][i],
    Yl: list of b x s blocks. Returns (logdet, G)."""
    logdet = 0.0
    G = 0.0
    D, F, Y = list(Dl), list(Fl), list(Yl)
    while True:
        m = len(D)
        if m == 1:
            L = numpy.linalg.cholesky(D[0])
            Z = scipy.linalg.solve_triangular(L, Y[0], lower=True)
            return logdet + 2 * numpy.sum(numpy.log(numpy.diag(L))), G + Z.T @ Z
        Wl, Wr, Zs = {}, {}, {}
        for i in range(1, m, 2):
            L = numpy.linalg.cholesky(D[i])
            logdet += 2 * numpy.sum(numpy.log(numpy.diag(L)))
            Wl[i] = scipy.linalg.solve_triangular(L, F[i - 1], lower=True)
            if i + 1 < m:
                Wr[i] = scipy.linalg.solve_triangular(L, F[i].T, lower=True)
            Zs[i] = scipy.linalg.solve_triangular(L, Y[i], lower=True)
            G = G + Zs[i].T @ Zs[i]
        D2, F2, Y2 = [], [], []
        for j in range(0, m, 2):
            d, y = D[j].copy(), Y[j].copy()
            if j - 1 >= 1:
                d -= Wr[j - 1].T @ Wr[j - 1]
                y -= Wr[j - 1].T @ Zs[j - 1]
            if j + 1 < m:
                d -= Wl[j + 1].T @ Wl[j + 1]
                y -= Wl[j + 1].T @ Zs[j + 1]
            D2.append(d)
            Y2.append(y)
            if j + 2 < m:
                F2.append(-Wr[j + 1].T @ Wl[j + 1])
        D, F, Y = D2, F2, Y2


if __name__ == '__main__':
    rng = numpy.random.RandomState(0)
    for nt in (1, 2, 3, 5, 8, 13, 16):
        b, s = 8, 3
        n = nt * b
        A = rng.randn(n, n)
        A = A @ A.T / n
        for i in range(n):       # keep the band (block tridiagonal, F upper triangular)
            for j in range(n):
                if abs(i // b - j // b) > 1 or (i // b == j // b + 1 and i % b > j % b) or \
                        (j // b == i // b + 1 and j % b > i % b):
                    A[i, j] = 0.0
        A += (n + 1.0) * numpy.eye(n) * 0.05 + numpy.eye(n) * numpy.abs(A).sum(1).max()
        Y = rng.randn(n, s)
        D = [A[i * b:(i + 1) * b, i * b:(i + 1) * b] for i in range(nt)]
        F = [A[(i + 1) * b:(i + 2) * b, i * b:(i + 1) * b] for i in range(nt - 1)]
        Yb = [Y[i * b:(i + 1) * b] for i in range(nt)]
        ld, G = bcr(D, F, Yb)
        ld_ref = numpy.linalg.slogdet(A)[1]
        G_ref = Y.T @ numpy.linalg.solve(A, Y)
        print(nt, abs(ld - ld_ref) / abs(ld_ref), numpy.max(numpy.abs(G - G_ref)) / numpy.max(numpy.abs(G_ref)))
