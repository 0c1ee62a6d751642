"""Dev prototype (numpy) of the band path's exact blocking, to validate the math
the HIP kernels implement (gpmi_band.hip): Householder panels of b columns with
the hh_col launch structure (partials S_j, nb2, pivot row), T by the forward
recurrence, the two-sided update W = X - 1/2 V (T^T V^T X), X = A V T, the
thin Q^T R transform, and the banded Cholesky per eta with C = E Linv^T."""
import sys

import numpy


def householder_panel(P):
    """In place: P (m x b) -> R (upper rows) and V below, as hh_col_kernel."""
    m, b = P.shape
    tau = numpy.zeros(b)
    for c in range(b):
        x0 = P[c, c]
        nb2 = numpy.sum(P[c + 1:, c] ** 2)
        S = P[c:, c] @ P[c:, c:]          # S_j for j >= c (S_c includes x0^2)
        if nb2 > 0:
            nrm = numpy.sqrt(x0 * x0 + nb2)
            alpha = -nrm if x0 >= 0 else nrm
            t = (alpha - x0) / alpha
            scale = 1.0 / (x0 - alpha)
            wv = (S[1:] - alpha * P[c, c + 1:]) * scale
            v = P[c:, c] * scale
            v[0] = 1.0
            P[c:, c + 1:] -= t * numpy.outer(v, wv)
            P[c + 1:, c] = v[1:]
            P[c, c] = alpha
            tau[c] = t
    return tau


def v_of(P):
    m, b = P.shape
    V = numpy.tril(P, -1)
    V[numpy.arange(b), numpy.arange(b)] = 1.0
    return V


def t_of(V, tau):
    b = V.shape[1]
    VtV = V.T @ V
    T = numpy.zeros((b, b))
    for c in range(b):
        T[:c, c] = -tau[c] * (T[:c, :c] @ VtV[:c, c])
        T[c, c] = tau[c]
    return T


def band_reduce(K, b):
    A = numpy.tril(K).copy()
    A = A + numpy.tril(A, -1).T   # full symmetric working copy (kernels keep lower + diag tiles)
    n = A.shape[0]
    Vs, Ts = [], []
    for j in range(n // b - 1):
        r0, c0 = (j + 1) * b, j * b
        P = A[r0:, c0:c0 + b]
        tau = householder_panel(P)
        V = v_of(P)
        T = t_of(V, tau)
        A22 = A[r0:, r0:]
        X = (A22 @ V) @ T
        Z = 0.5 * (T.T @ (V.T @ X))
        W = X - V @ Z
        A22 -= W @ V.T + V @ W.T
        Vs.append(V.copy())
        Ts.append(T)
    return A, Vs, Ts


def apply_qt(Vs, Ts, R, b):
    R = R.copy()
    for j, (V, T) in enumerate(zip(Vs, Ts)):
        r0 = (j + 1) * b
        R[r0:] -= V @ (T.T @ (V.T @ R[r0:]))
    return R


def band_chol(A, b, eta, Y, n):
    N = A.shape[0]
    nt = N // b
    ld, G = 0.0, numpy.zeros((Y.shape[1], Y.shape[1]))
    D = A[:b, :b] + eta * numpy.eye(b)
    r = Y[:b].copy()
    for k in range(nt):
        L = numpy.linalg.cholesky(D)
        Li = numpy.linalg.inv(L)
        idx = numpy.arange(k * b, (k + 1) * b) < n
        ld += 2 * numpy.sum(numpy.log(numpy.diag(L))[idx])
        y = Li @ r
        G += y.T @ y
        if k + 1 == nt:
            break
        E = numpy.triu(A[(k + 1) * b:(k + 2) * b, k * b:(k + 1) * b])
        C = E @ Li.T
        r = Y[(k + 1) * b:(k + 2) * b] - C @ y
        D = A[(k + 1) * b:(k + 2) * b, (k + 1) * b:(k + 2) * b] + eta * numpy.eye(b) - C @ C.T
    return ld, G


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    N = (n + b - 1) // b * b
    rng = numpy.random.RandomState(0)
    pts = rng.rand(n, 2)
    d = numpy.sqrt(((pts[:, None, :] - pts[None, :, :]) ** 2).sum(-1)) / 0.1
    K = (1 + numpy.sqrt(3) * d) * numpy.exp(-numpy.sqrt(3) * d)
    Kp = numpy.eye(N)
    Kp[:n, :n] = K
    R = numpy.zeros((N, 4))
    R[:n] = rng.randn(n, 4)
    A, Vs, Ts = band_reduce(Kp, b)
    Y = apply_qt(Vs, Ts, R, b)
    for eta in (1e-3, 0.1, 1.0, 10.0):
        ld, G = band_chol(A, b, eta, Y, n)
        M = K + eta * numpy.eye(n)
        s, ld_ref = numpy.linalg.slogdet(M)
        G_ref = R[:n].T @ numpy.linalg.solve(M, R[:n])
        print('eta %-6g logdet rel %.2e  gram rel %.2e' % (
            eta, abs(ld - ld_ref) / abs(ld_ref),
            numpy.abs(G - G_ref).max() / numpy.abs(G_ref).max()))


if __name__ == '__main__':
    main()
