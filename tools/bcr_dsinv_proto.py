"""numpy prototype: trace((B + eta I)^-2) of a block-tridiagonal B without
eigenvalues, as -d/deta trace((B + eta I)^-1), by forward-mode differentiation
(tangent d/deta carried beside every block) of the block cyclic reduction factor
and of the selected inversion of tools/bcr_sinv_proto.py (gpmi_bcr.hip).

Factor, per level, eliminated (odd) block p with tangent dD_p (level 0: I):
    M_p      = Phi(Linv_p dD_p Linv_p^T)        Phi: strict lower + half diagonal
    dLinv_p  = -M_p Linv_p                      (S = L L^T, dS = dL L^T + L dL^T)
    dW_l     = dLinv_p F_{p-1} + Linv_p dF_{p-1}
    dW_r     = dLinv_p F_p^T   + Linv_p dF_p^T
  even j:
    dD_j'    = dD_j - (dW_r^T W_r + W_r^T dW_r)(j-1) - (dW_l^T W_l + W_l^T dW_l)(j+1)
    dF_j/2'  = -(dW_r^T W_l + W_r^T dW_l)(j+1)
Selected inversion, top-down:
    dX_s     = dW_s^T Linv_p + W_s^T dLinv_p
    dZ_sp    = -(dZ_sl X_l + Z_sl dX_l + dZ_sr X_r + Z_sr dX_r)
    dZ_pp    = dLinv_p^T Linv_p + Linv_p^T dLinv_p - dX_l^T Z_lp - X_l^T dZ_lp
               - dX_r^T Z_rp - X_r^T dZ_rp
    trace(S^-2) = -sum_p trace(dZ_pp).
Run: python tools/bcr_dsinv_proto.py   (prints nt, rel. error of tr(S^-1), of
tr(S^-2) against numpy, and the largest diagonal-block error of dZ = -S^-2)."""
import numpy as np


def phi(M):
    return np.tril(M, -1) + 0.5 * np.diag(np.diag(M))


def bcr_factor_tan(D, F):
    nt = len(D)
    b = D[0].shape[0]
    Linv = [None] * nt
    dLinv = [None] * nt
    W = [[None, None] for _ in range(nt)]
    dW = [[None, None] for _ in range(nt)]
    Dl, Fl = list(D), list(F)
    dDl = [np.eye(b) for _ in range(nt)]
    dFl = [np.zeros((b, b)) for _ in range(nt - 1)]
    m, lvl, ms = nt, 0, []
    while m > 1:
        ms.append(m)
        for p in range(1, m, 2):
            o = p << lvl
            Li = np.linalg.inv(np.linalg.cholesky(Dl[p]))
            Linv[o] = Li
            dLi = -phi(Li @ dDl[p] @ Li.T) @ Li
            dLinv[o] = dLi
            W[o][0] = Li @ Fl[p - 1]
            dW[o][0] = dLi @ Fl[p - 1] + Li @ dFl[p - 1]
            if p + 1 < m:
                W[o][1] = Li @ Fl[p].T
                dW[o][1] = dLi @ Fl[p].T + Li @ dFl[p].T
        D2, F2, dD2, dF2 = [], [], [], []
        for j in range(0, m, 2):
            Dj, dDj = Dl[j].copy(), dDl[j].copy()
            if j >= 1:
                Wr, dWr = W[(j - 1) << lvl][1], dW[(j - 1) << lvl][1]
                Dj -= Wr.T @ Wr
                dDj -= dWr.T @ Wr + Wr.T @ dWr
            if j + 1 < m:
                Wl, dWl = W[(j + 1) << lvl][0], dW[(j + 1) << lvl][0]
                Dj -= Wl.T @ Wl
                dDj -= dWl.T @ Wl + Wl.T @ dWl
            D2.append(Dj)
            dD2.append(dDj)
            if j + 2 < m:
                o1 = (j + 1) << lvl
                F2.append(-W[o1][1].T @ W[o1][0])
                dF2.append(-(dW[o1][1].T @ W[o1][0] + W[o1][1].T @ dW[o1][0]))
        Dl, Fl, dDl, dFl = D2, F2, dD2, dF2
        m = (m + 1) // 2
        lvl += 1
    Li = np.linalg.inv(np.linalg.cholesky(Dl[0]))
    Linv[0] = Li
    dLinv[0] = -phi(Li @ dDl[0] @ Li.T) @ Li
    return Linv, dLinv, W, dW, ms, lvl


def sinv_tan(Linv, dLinv, W, dW, ms, L):
    nt = len(Linv)
    Zd, dZd = [None] * nt, [None] * nt
    Zo = [[None, None] for _ in range(nt)]
    dZo = [[None, None] for _ in range(nt)]
    Zd[0] = Linv[0].T @ Linv[0]
    dZd[0] = dLinv[0].T @ Linv[0] + Linv[0].T @ dLinv[0]
    for lvl in range(L - 1, -1, -1):
        m = ms[lvl]
        for p in range(1, m, 2):
            o, ol = p << lvl, (p - 1) << lvl
            Li, dLi = Linv[o], dLinv[o]
            Xl = W[o][0].T @ Li
            dXl = dW[o][0].T @ Li + W[o][0].T @ dLi
            right = p + 1 < m
            if right:
                orr = (p + 1) << lvl
                Xr = W[o][1].T @ Li
                dXr = dW[o][1].T @ Li + W[o][1].T @ dLi
                lp = (p - 1) // 2
                if (lp + 1) % 2 == 1:
                    Zlr, dZlr = Zo[orr][0], dZo[orr][0]
                else:
                    Zlr, dZlr = Zo[ol][1].T, dZo[ol][1].T
                Zlp = -(Zd[ol] @ Xl + Zlr @ Xr)
                Zrp = -(Zlr.T @ Xl + Zd[orr] @ Xr)
                dZlp = -(dZd[ol] @ Xl + Zd[ol] @ dXl + dZlr @ Xr + Zlr @ dXr)
                dZrp = -(dZlr.T @ Xl + Zlr.T @ dXl + dZd[orr] @ Xr + Zd[orr] @ dXr)
                Zo[o], dZo[o] = [Zlp, Zrp], [dZlp, dZrp]
                Zd[o] = Li.T @ Li - Xl.T @ Zlp - Xr.T @ Zrp
                dZd[o] = dLi.T @ Li + Li.T @ dLi - dXl.T @ Zlp - Xl.T @ dZlp \
                    - dXr.T @ Zrp - Xr.T @ dZrp
            else:
                Zlp = -(Zd[ol] @ Xl)
                dZlp = -(dZd[ol] @ Xl + Zd[ol] @ dXl)
                Zo[o], dZo[o] = [Zlp, None], [dZlp, None]
                Zd[o] = Li.T @ Li - Xl.T @ Zlp
                dZd[o] = dLi.T @ Li + Li.T @ dLi - dXl.T @ Zlp - Xl.T @ dZlp
    return (sum(np.trace(z) for z in Zd), -sum(np.trace(z) for z in dZd), dZd)


def main():
    rng = np.random.RandomState(1)
    for nt in (1, 2, 3, 5, 8, 11, 16, 17):
        b = 6
        n = nt * b
        A = np.zeros((n, n))
        for i in range(nt):
            M = rng.randn(b, b)
            A[i*b:(i+1)*b, i*b:(i+1)*b] = M @ M.T + 0.5 * np.eye(b)
            if i + 1 < nt:
                Fi = np.triu(rng.randn(b, b)) * 0.5
                A[(i+1)*b:(i+2)*b, i*b:(i+1)*b] = Fi
                A[i*b:(i+1)*b, (i+1)*b:(i+2)*b] = Fi.T
        lam = np.linalg.eigvalsh(A)
        A += (0.1 - lam[0]) * np.eye(n)      # SPD, moderately conditioned
        D = [A[i*b:(i+1)*b, i*b:(i+1)*b] for i in range(nt)]
        F = [A[(i+1)*b:(i+2)*b, i*b:(i+1)*b] for i in range(nt - 1)]
        fac = bcr_factor_tan(D, F)
        t1, t2, dZd = sinv_tan(*fac)
        Ai = np.linalg.inv(A)
        A2 = Ai @ Ai
        e1 = abs(t1 - np.trace(Ai)) / np.trace(Ai)
        e2 = abs(t2 - np.trace(A2)) / np.trace(A2)
        dz = max(np.abs(dZd[i] + A2[i*b:(i+1)*b, i*b:(i+1)*b]).max() for i in range(nt))
        print(nt, '%.2e %.2e %.2e' % (e1, e2, dz))


if __name__ == '__main__':
    main()
