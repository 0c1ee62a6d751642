"""Host prototype of chase_systolic_kernel (gpmi_chase.hip): the same per-position
state (D, E in circular physical layout), messages and window slide, run
sequentially in an order the hand-offs allow (per sweep: steps 1-4 for k = 0..K-1,
then every slide). Checks the tridiagonal's eigenvalues against numpy for small b.
Development tool; not used by the tests or the product path."""
import numpy


def dlarfg(x0, nb2):
    if nb2 > 0:
        nrm = numpy.sqrt(x0 * x0 + nb2)
        beta = -nrm if x0 >= 0 else nrm
        return (beta - x0) / beta, beta, 1.0 / (x0 - beta)
    return 0.0, x0, 0.0


def chase(Bfull, b):
    n = Bfull.shape[0]
    M = b - 1
    K = (n - 1 + b - 1) // b
    A = lambda r, c: Bfull[max(r, c), min(r, c)] if (r < n and c < n and abs(r - c) <= b) else 0.0
    D = [numpy.zeros((b, b)) for _ in range(K)]
    E = [numpy.zeros((b, b)) for _ in range(K)]
    for k in range(K):
        rb = 1 + k * b
        for i in range(b):
            for j in range(b):
                D[k][i, j] = A(rb + i, rb + j)
                E[k][i, j] = A(rb + b + i, rb + j)
    xk0 = numpy.array([A(1 + i, 0) for i in range(b)])
    d = numpy.zeros(n)
    e2 = numpy.zeros(n)
    d[0] = Bfull[0, 0]
    s_end = [min(n - 3, n - 2 - k * b) for k in range(K)]
    R = {}
    C = {}
    for s in range(n - 2):
        off = s & M
        act = [k for k in range(K) if s <= s_end[k]]
        for k in act:
            nxt = s + 1 + (k + 1) * b < n
            sv = numpy.zeros(b)
            if k == 0:
                tau, beta, sc = dlarfg(xk0[0], numpy.sum(xk0[1:] ** 2))
                for i in range(b):
                    sv[(i + off) & M] = 1.0 if i == 0 else xk0[i] * sc
                e2[s] = beta * beta
            else:
                vlog, tau = R[(s, k)]
                for i in range(b):
                    sv[(i + off) & M] = vlog[i]
            Dk, Ek = D[k], E[k]
            if tau != 0:
                p = tau * (Dk @ sv)
                q = tau * (Ek @ sv)
                vp = p @ sv
                w = p - 0.5 * tau * vp * sv
                Dk -= numpy.outer(sv, w) + numpy.outer(w, sv)
                Ek -= numpy.outer(q, sv)
            if nxt:
                sx = Ek[:, off].copy()
                x0 = sx[off]
                nb2 = numpy.sum(sx ** 2) - x0 * x0
                taun, betan, scn = dlarfg(x0, nb2)
                sv2 = sx * scn
                sv2[off] = 1.0
                R[(s, k + 1)] = (numpy.array([1.0 if i == 0 else sx[(i + off) & M] * scn
                                              for i in range(b)]), taun)
                if taun != 0:
                    r = taun * (Ek.T @ sv2)
                    Ek -= numpy.outer(sv2, r)
                    Ek[:, off] = 0.0
                    Ek[off, off] = betan
            scol = Dk[:, off].copy()
            e00 = Ek[off, off]
            if k >= 1:
                C[(s, k)] = (numpy.array([scol[(i + off) & M] for i in range(b)]), e00)
            else:
                d[s + 1] = scol[off]
                xk0 = numpy.array([scol[(i + 1 + off) & M] for i in range(b - 1)] + [e00])
                if s == n - 3:
                    o1 = (off + 1) & M
                    e2[n - 2] = scol[o1] ** 2
                    d[n - 1] = Dk[o1, o1]
        for k in act:
            nxt = s + 1 + (k + 1) * b < n
            Dk, Ek = D[k], E[k]
            serow = Ek[off, :].copy()
            snew, ne00 = C[(s, k + 1)] if nxt else (numpy.zeros(b), 0.0)
            Dk[off, :] = serow
            Dk[:, off] = serow
            Dk[off, off] = snew[0]
            Ek[off, :] = 0.0
            for r in range(b):
                if r != off:
                    Ek[r, off] = snew[((r - off - 1) & M) + 1]
            Ek[off, off] = ne00
    return d, e2


if __name__ == '__main__':
    rng = numpy.random.RandomState(0)
    for n, b in ((37, 4), (64, 8), (50, 8), (9, 4), (3, 4), (130, 16), (129, 8)):
        X = rng.randn(n, n)
        S = X + X.T
        # banded symmetric
        Bm = numpy.where(numpy.abs(numpy.subtract.outer(numpy.arange(n), numpy.arange(n))) <= b, S, 0.0)
        d, e2 = chase(numpy.tril(Bm), b)
        T = numpy.diag(d) + numpy.diag(numpy.sqrt(e2[:-1]), 1) + numpy.diag(numpy.sqrt(e2[:-1]), -1)
        lt = numpy.linalg.eigvalsh(T)
        lb = numpy.linalg.eigvalsh(Bm)
        print(n, b, numpy.max(numpy.abs(lt - lb)) / numpy.max(numpy.abs(lb)))


def chase_split(Bfull, b):
    """The same chase with each position split into a D workgroup (D_k) and an E
    workgroup (E_k) that exchange only messages: R (reflector, E(k-1) -> E(k), D(k);
    position 0's from D(0)), Dcol (D(k)'s first column after H D H -> E(k-1), and its
    first entry -> D(k-1)), Erow (E(k)'s first row after both updates -> D(k)),
    E00 (E(k)[0][0] = beta' -> E(k-1); for k = 0 -> D(0), the last entry of the next
    sweep's column)."""
    n = Bfull.shape[0]
    M = b - 1
    K = (n - 1 + b - 1) // b
    A = lambda r, c: Bfull[max(r, c), min(r, c)] if (r < n and c < n and abs(r - c) <= b) else 0.0
    D = [numpy.zeros((b, b)) for _ in range(K)]
    E = [numpy.zeros((b, b)) for _ in range(K)]
    for k in range(K):
        rb = 1 + k * b
        for i in range(b):
            for j in range(b):
                D[k][i, j] = A(rb + i, rb + j)
                E[k][i, j] = A(rb + b + i, rb + j)
    d = numpy.zeros(n)
    e2 = numpy.zeros(n)
    d[0] = Bfull[0, 0]
    s_end = [min(n - 3, n - 2 - k * b) for k in range(K)]
    R, Dcol, Erow, E00 = {}, {}, {}, {}
    xk = numpy.array([A(1 + i, 0) for i in range(b)])   # D(0)'s column of sweep 0
    for s in range(n - 2):
        off = s & M
        act = [k for k in range(K) if s <= s_end[k]]
        # D(0): the reflector of sweep s from its column
        if s > 0:
            xk = numpy.append(Dcol[(s - 1, 0)][1:], E00[(s - 1, 0)])
        tau, beta, sc = dlarfg(xk[0], numpy.sum(xk[1:] ** 2))
        R[(s, 0)] = (numpy.array([1.0] + list(xk[1:] * sc)), tau)
        e2[s] = beta * beta
        for k in act:
            nxt = s + 1 + (k + 1) * b < n
            vlog, tau = R[(s, k)]
            sv = numpy.zeros(b)
            for i in range(b):
                sv[(i + off) & M] = vlog[i]
            # D(k)
            Dk = D[k]
            if tau != 0:
                p = tau * (Dk @ sv)
                vp = p @ sv
                w = p - 0.5 * tau * vp * sv
                Dk -= numpy.outer(sv, w) + numpy.outer(w, sv)
            Dcol[(s, k)] = numpy.array([Dk[(i + off) & M, off] for i in range(b)])
            if k == 0:
                d[s + 1] = Dk[off, off]
                if s == n - 3:
                    o1 = (off + 1) & M
                    e2[n - 2] = Dk[o1, off] ** 2
                    d[n - 1] = Dk[o1, o1]
            # E(k)
            Ek = E[k]
            if tau != 0:
                q = tau * (Ek @ sv)
                Ek -= numpy.outer(q, sv)
            betan = 0.0
            if nxt:
                sx = Ek[:, off].copy()
                x0 = sx[off]
                taun, betan, scn = dlarfg(x0, numpy.sum(sx ** 2) - x0 * x0)
                sv2 = sx * scn
                sv2[off] = 1.0
                R[(s, k + 1)] = (numpy.array([1.0 if i == 0 else sx[(i + off) & M] * scn
                                              for i in range(b)]), taun)
                if taun != 0:
                    r = taun * (Ek.T @ sv2)
                    Ek -= numpy.outer(sv2, r)
                    Ek[:, off] = 0.0
                    Ek[off, off] = betan
            Erow[(s, k)] = Ek[off, :].copy()
            E00[(s, k)] = betan
        for k in act:
            nxt = s + 1 + (k + 1) * b < n
            dn = Dcol[(s, k + 1)] if nxt else numpy.zeros(b)
            en = E00[(s, k + 1)] if nxt else 0.0
            Dk, Ek = D[k], E[k]
            serow = Erow[(s, k)]
            Dk[off, :] = serow
            Dk[:, off] = serow
            Dk[off, off] = dn[0]
            Ek[off, :] = 0.0
            for r in range(b):
                if r != off:
                    Ek[r, off] = dn[((r - off - 1) & M) + 1]
            Ek[off, off] = en
    return d, e2


if __name__ == '__main__':
    rng = numpy.random.RandomState(1)
    for n, b in ((37, 4), (64, 8), (9, 4), (3, 4), (129, 8)):
        X = rng.randn(n, n)
        S = X + X.T
        Bm = numpy.where(numpy.abs(numpy.subtract.outer(numpy.arange(n), numpy.arange(n))) <= b, S, 0.0)
        d, e2 = chase_split(numpy.tril(Bm), b)
        T = numpy.diag(d) + numpy.diag(numpy.sqrt(e2[:-1]), 1) + numpy.diag(numpy.sqrt(e2[:-1]), -1)
        print('split', n, b, numpy.max(numpy.abs(numpy.linalg.eigvalsh(T) - numpy.linalg.eigvalsh(Bm)))
              / numpy.max(numpy.abs(numpy.linalg.eigvalsh(Bm))))
