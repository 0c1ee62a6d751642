"""Dev prototype (numpy) of a communication-avoiding panel for the band reduction:
shifted CholeskyQR3 (Fukaya et al., SIAM J. Sci. Comput. 42 (2020) A477) of the
m x b panel, then Householder reconstruction (Ballard et al., IPDPS 2014:
LU without pivoting of Q - [S; 0], S_ii = -sign of the running pivot) to get the
compact-WY V, T the rest of the reduction consumes. Compares the band spectrum /
logdet with numpy and prints each panel's orthogonality and conditioning, so the
device kernels can be checked against it. Usage: cholqr_proto.py [grid] [nu]"""
import sys

import numpy

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from band_proto import v_of, t_of, householder_panel  # noqa: E402

U_RND = 2.0 ** -53


FO_TAU = (0.0, 1e-4, 3e-8)   # first-order thresholds on ||G - I||_F (gpmi_band_api.hip)


def cholqr_panel(P, shifted_passes=1, passes=3, first_order=True):
    """Return (V, tau, R_hh, info) with (I - V T V^T)^T P = [R_hh; 0], or None.
    A pass whose Gram is within FO_TAU of I applies the first-order factor
    Linv = I - E_l (E_l = stril(E) + diag(E) / 2) instead of a Cholesky, and
    records L = Linv^-1 (as cq_chol_kernel / cq_top_kernel)."""
    m, b = P.shape
    Q = P.copy()
    R = numpy.eye(b)
    info = {'first_order': []}
    for k in range(passes):
        G = Q.T @ Q
        if k < shifted_passes:
            s = 11.0 * (m * b + b * (b + 1)) * U_RND * numpy.trace(G)
            G = G + s * numpy.eye(b)
        E = G - numpy.eye(b)
        if first_order and k > 0 and numpy.linalg.norm(E) <= FO_TAU[min(k, 2)]:
            El = numpy.tril(E, -1) + 0.5 * numpy.diag(numpy.diag(E))
            Linv = numpy.eye(b) - El
            L = numpy.linalg.inv(Linv)
            info['first_order'].append(k)
        else:
            try:
                L = numpy.linalg.cholesky(G)
            except numpy.linalg.LinAlgError:
                info['fail'] = k
                return None, info
            Linv = numpy.linalg.inv(L)
        Q = Q @ Linv.T
        R = L.T @ R
    info['orth'] = numpy.linalg.norm(Q.T @ Q - numpy.eye(b))
    info['resid'] = numpy.linalg.norm(P - Q @ R) / numpy.linalg.norm(P)
    # Householder reconstruction: LU (no pivoting) of Q - [S; 0]
    A = Q.copy()
    S = numpy.zeros(b)
    for i in range(b):
        S[i] = -1.0 if A[i, i] >= 0 else 1.0
        A[i, i] -= S[i]
        A[i + 1:, i] /= A[i, i]
        A[i + 1:, i + 1:] -= numpy.outer(A[i + 1:, i], A[i, i + 1:])
    Uu = numpy.triu(A[:b])
    V = numpy.tril(A, -1)
    V[numpy.arange(b), numpy.arange(b)] = 1.0
    tau = -numpy.diag(Uu) * S
    Rhh = S[:, None] * R
    return (V, tau, Rhh), info


def band_reduce_cholqr(K, b, stats):
    A = numpy.tril(K).copy()
    A = A + numpy.tril(A, -1).T
    n = A.shape[0]
    for j in range(n // b - 1):
        r0, c0 = (j + 1) * b, j * b
        P = A[r0:, c0:c0 + b]
        out, info = cholqr_panel(P)
        if out is None:
            tau = householder_panel(P)
            V = v_of(P)
            stats.append(('hh', info))
        else:
            V, tau, Rhh = out
            P[:] = 0.0
            P[:b] = Rhh
            stats.append(('cq', info))
        T = t_of(V, tau)
        A22 = A[r0:, r0:]
        X = (A22 @ V) @ T
        Z = 0.5 * (T.T @ (V.T @ X))
        W = X - V @ Z
        A22 -= W @ V.T + V @ W.T
        # keep the band only (the panel's entries below R are the reflectors' zeros)
        A[c0:c0 + b, r0:] = A[r0:, c0:c0 + b].T
    return A


def main():
    grid = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    nu = float(sys.argv[2]) if len(sys.argv) > 2 else 1.5
    b = 128
    x = numpy.linspace(0, 1, grid)
    pts = numpy.array([(a, c) for a in x for c in x])
    d = numpy.sqrt(((pts[:, None, :] - pts[None, :, :]) ** 2).sum(-1)) / 0.1
    if nu == 1.5:
        K = (1 + numpy.sqrt(3) * d) * numpy.exp(-numpy.sqrt(3) * d)
    elif nu == 2.5:
        K = (1 + numpy.sqrt(5) * d + 5 * d * d / 3) * numpy.exp(-numpy.sqrt(5) * d)
    elif nu == 0.5:
        K = numpy.exp(-d)
    else:
        K = numpy.exp(-0.5 * d * d)
    n = K.shape[0]
    stats = []
    A = band_reduce_cholqr(K, b, stats)
    B = numpy.tril(numpy.triu(A, -b), b)
    ev = numpy.linalg.eigvalsh(B)
    ev_ref = numpy.linalg.eigvalsh(K)
    print('n %d nu %s: panels cholqr %d / householder %d' % (
        n, nu, sum(s[0] == 'cq' for s in stats), sum(s[0] == 'hh' for s in stats)))
    orth = [s[1]['orth'] for s in stats if s[0] == 'cq']
    res = [s[1]['resid'] for s in stats if s[0] == 'cq']
    if orth:
        print('max orth %.2e  max resid %.2e' % (max(orth), max(res)))
    print('eig max abs err / |K| %.2e' % (numpy.abs(ev - ev_ref).max() / ev_ref.max()))
    for eta in (1e-3, 1.0):
        ld = numpy.linalg.slogdet(B + eta * numpy.eye(n))[1]
        ld_ref = numpy.linalg.slogdet(K + eta * numpy.eye(n))[1]
        print('eta %g logdet rel err %.2e' % (eta, abs(ld - ld_ref) / abs(ld_ref)))


if __name__ == '__main__':
    main()
