"""numpy prototype: trace((B + eta I)^-1) of a block-tridiagonal B from its block
cyclic reduction factor (gpmi_bcr.hip) by selected inversion down the reduction
tree (Takahashi, Fagan and Chin 1973; Erisman and Tinney 1975): per eliminated
block p of level l with parents l = p - 1, r = p + 1 (even blocks of level l),
    X_s  = W_s^T Linv_p                     (L_{s,p} L_pp^-1)
    Z_sp = -(Z_sl X_l + Z_sr X_r)            s in {l, r}
    Z_pp = Linv_p^T Linv_p - X_l^T Z_lp - X_r^T Z_rp
top-down from the last level's single block (Z = Linv^T Linv). Z_lr of the parents
is the off-diagonal block their own elimination produced one level up.
Run: python tools/bcr_sinv_proto.py   (prints the relative trace error)."""
import numpy as np


def bcr_factor(D, F):
    """D[i] diagonal blocks, F[i] = A_{i+1,i}. Returns per original index o:
    Linv[o], W[o] = (W_l, W_r) and the level sizes."""
    nt = len(D)
    b = D[0].shape[0]
    Linv = [None] * nt
    W = [[None, None] for _ in range(nt)]
    Dl, Fl = list(D), list(F)
    m, lvl, ms = nt, 0, []
    while m > 1:
        ms.append(m)
        for p in range(1, m, 2):
            o = p << lvl
            L = np.linalg.cholesky(Dl[p])
            Li = np.linalg.inv(L)
            Linv[o] = Li
            W[o][0] = Li @ Fl[p - 1]
            W[o][1] = Li @ Fl[p].T if p + 1 < m else None
        D2, F2 = [], []
        for j in range(0, m, 2):
            o = j << lvl
            Dj = Dl[j].copy()
            if j >= 1:
                Wr = W[(j - 1) << lvl][1]
                Dj -= Wr.T @ Wr
            if j + 1 < m:
                Wl = W[(j + 1) << lvl][0]
                Dj -= Wl.T @ Wl
            D2.append(Dj)
            if j + 2 < m:
                Wl = W[(j + 1) << lvl][0]
                Wr = W[(j + 1) << lvl][1]
                F2.append(-Wr.T @ Wl)
        Dl, Fl = D2, F2
        m = (m + 1) // 2
        lvl += 1
    L = np.linalg.cholesky(Dl[0])
    Linv[0] = np.linalg.inv(L)
    return Linv, W, ms, lvl


def sinv_trace(Linv, W, ms, L):
    nt = len(Linv)
    Zd = [None] * nt
    Zo = [[None, None] for _ in range(nt)]
    Zd[0] = Linv[0].T @ Linv[0]
    for lvl in range(L - 1, -1, -1):
        m = ms[lvl]
        for p in range(1, m, 2):
            o, ol = p << lvl, (p - 1) << lvl
            right = p + 1 < m
            Xl = W[o][0].T @ Linv[o]
            if right:
                orr = (p + 1) << lvl
                Xr = W[o][1].T @ Linv[o]
                lp = (p - 1) // 2          # parents' indices one level up
                if (lp + 1) % 2 == 1:      # r' odd: its left-parent block
                    Zlr = Zo[orr][0]
                else:                      # l' odd: its right-parent block, transposed
                    Zlr = Zo[ol][1].T
                Zlp = -(Zd[ol] @ Xl + Zlr @ Xr)
                Zrp = -(Zlr.T @ Xl + Zd[orr] @ Xr)
                Zo[o] = [Zlp, Zrp]
                Zd[o] = Linv[o].T @ Linv[o] - Xl.T @ Zlp - Xr.T @ Zrp
            else:
                Zlp = -(Zd[ol] @ Xl)
                Zo[o] = [Zlp, None]
                Zd[o] = Linv[o].T @ Linv[o] - Xl.T @ Zlp
    return sum(np.trace(z) for z in Zd), Zd


def main():
    rng = np.random.RandomState(1)
    for nt in (1, 2, 3, 5, 8, 11, 16, 17):
        b = 6
        n = nt * b
        A = np.zeros((n, n))
        for i in range(nt):
            M = rng.randn(b, b)
            A[i*b:(i+1)*b, i*b:(i+1)*b] = M @ M.T + b * np.eye(b)
            if i + 1 < nt:
                Fi = np.triu(rng.randn(b, b)) * 0.5
                A[(i+1)*b:(i+2)*b, i*b:(i+1)*b] = Fi
                A[i*b:(i+1)*b, (i+1)*b:(i+2)*b] = Fi.T
        D = [A[i*b:(i+1)*b, i*b:(i+1)*b] for i in range(nt)]
        F = [A[(i+1)*b:(i+2)*b, i*b:(i+1)*b] for i in range(nt - 1)]
        Linv, W, ms, L = bcr_factor(D, F)
        tr, Zd = sinv_trace(Linv, W, ms, L)
        Ai = np.linalg.inv(A)
        ex = np.trace(Ai)
        dz = max(np.abs(Zd[i] - Ai[i*b:(i+1)*b, i*b:(i+1)*b]).max() for i in range(nt))
        print(nt, abs(tr - ex) / abs(ex), dz)


if __name__ == '__main__':
    main()
