"""numpy prototype of the delayed CGS2 (DCGS2) Lanczos of the sparse path (dev
tool): per step ONE dots pass over the basis (the lagged second pass of u_k
and the projections of y = A u_k together) and ONE update pass (v_k and
u_{k+1} written together), against oracle.sparse.lanczos (CGS2: four basis
passes per step). Low-synchronisation Gram-Schmidt with delayed
reorthogonalisation: Bielich, Langou, Thomas, Swirydowicz, Yamazaki, Boman,
Parallel Computing 112 (2022) 102940.

Step k (V = [v_0 .. v_{k-1}] final, u_k projected once, H the Hessenberg
columns so far, A V = V_{k+1} H):
  y = A u_k
  dots:   s = V^T u_k, t = V^T y, sig = u_k.u_k, tau = u_k.y
  rho = sqrt(sig - s.s)                 (beta_{k-1}, final)
  H[:, k-1] += s                        (alpha_{k-1}, beta_{k-2} final)
  v_k = (u_k - V s) / rho
  A v_k = (y - V_{k+1} H s) / rho  ->  h = V_{k+1}^T A v_k from (t, tau) and H s
  update: u_{k+1} = A v_k - V_{k+1} h   (v_k formed in the same pass)
"""
import sys
import numpy

sys.path.insert(0, '.')
from oracle import sparse as osp  # noqa: E402


def lanczos_dcgs2(K, v0, steps):
    n = v0.shape[0]
    V = numpy.zeros((steps + 1, n))
    H = numpy.zeros((steps + 2, steps + 1))   # H[i, j] = coefficient of v_i in A v_j
    u = v0 / numpy.linalg.norm(v0)
    # step 0: v_0 = u exactly normalised, no lag yet
    V[0] = u
    y = K @ u
    h0 = numpy.dot(u, y)
    H[0, 0] = h0
    u = y - h0 * V[0]
    alpha, beta = [], []
    for k in range(1, steps + 1):
        y = K @ u
        Vk = V[:k]
        s = Vk @ u
        t = Vk @ y
        sig = numpy.dot(u, u)
        tau = numpy.dot(u, y)
        rho = numpy.sqrt(sig - numpy.dot(s, s))
        H[:k, k - 1] += s
        H[k, k - 1] = rho
        # alpha_{k-1}, beta_{k-1} are final now
        a_prev = H[k - 1, k - 1]
        alpha.append(a_prev)
        if k == steps or not rho > 1e-13 * max(1.0, abs(a_prev)):
            break
        beta.append(rho)
        Hs = H[:k + 1, :k] @ s                  # A V_k s = V_{k+1} H s
        # h = V_{k+1}^T A v_k
        h = numpy.zeros(k + 1)
        h[:k] = (t - Hs[:k]) / rho
        h[k] = (tau - numpy.dot(s, t)) / rho ** 2 - Hs[k] / rho
        vk = (u - Vk.T @ s) / rho
        V[k] = vk
        u = (y - V[:k + 1].T @ Hs) / rho - V[:k + 1].T @ h
        H[:k + 1, k] = h
    return numpy.array(alpha), numpy.array(beta)


if __name__ == '__main__':
    import scipy.sparse
    rng = numpy.random.RandomState(0)
    pts = rng.rand(4000, 2)
    K = osp.sparse_correlation(pts, 0.03, 1.5, 0.01)[0]
    K = (K + 0.3 * scipy.sparse.identity(K.shape[0])).tocsr()
    P = osp.rademacher_probes(K.shape[0], 4, 0)
    for p in range(4):
        a1, b1 = osp.lanczos(K, P[:, p], 30)
        a2, b2 = lanczos_dcgs2(K, P[:, p], 30)
        k = min(a1.size, a2.size)
        ra = numpy.max(numpy.abs(a1[:k] - a2[:k]) / numpy.abs(a1[:k]))
        rb = numpy.max(numpy.abs(b1[:k - 1] - b2[:k - 1]) / numpy.abs(b1[:k - 1]))
        t1, w1 = osp.slq_nodes(a1, b1)
        t2, w2 = osp.slq_nodes(a2[:a1.size], b2[:a1.size - 1])
        ld1 = numpy.sum(w1 * numpy.log(t1 + 1.0))
        ld2 = numpy.sum(w2 * numpy.log(t2 + 1.0))
        print(p, a1.size, a2.size, 'alpha rel %.2e beta rel %.2e quad rel %.2e'
              % (ra, rb, abs(ld1 - ld2) / abs(ld1)))
