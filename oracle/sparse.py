"""Tapered (sparse) Matérn correlation and the stochastic Lanczos quadrature
(oracle restatement; TEST INFRASTRUCTURE ONLY).

Assembly restates /root/reference/gaussian_proc/generate_correlation/
_generate_sparse_correlation.pyx with the two argument fixes SURVEY §0.4 lists
(the shipped file raises TypeError before doing any work):
  gamma_function              :208-233
  _ball_radius / _ball_volume :240-287   (_ball_volume(r) -> _ball_volume(r, dimension), :390)
  _estimate_kernel_threshold  :294-413
  _estimate_max_nnz           :420-465   (called with 3 args at :542 -> 4 args)
  _generate_correlation_matrix :35-201   (keep K_ij > threshold, i <= j, mirrored)

SLQ restates the published stochastic Lanczos quadrature that imate's 'slq'
method implements (imate is absent: parity unpinned against imate itself; the
device path is checked against this restatement with identical probes, and
against exact logdet / traceinv within Monte-Carlo error):
  logdet(K + eta I)   ~= n/s sum_probes sum_i tau_i^2 log(theta_i + eta)
  tr((K + eta I)^-p)  ~= n/s sum_probes sum_i tau_i^2 (theta_i + eta)^-p
with (theta_i, tau_i) the Ritz values / first eigenvector components of the
Lanczos tridiagonal of K started at the normalised Rademacher probe. One
Lanczos run per probe serves every eta (the Krylov space of K + eta I does not
depend on eta).
"""

import numpy
import scipy.sparse

from .matern import matern_kernel, broadcast_scale, scaled_distance


def gamma_function(dimension):
    """Gamma(dimension/2 + 1), :208-233."""
    if dimension % 2 == 0:
        k = 0.5 * dimension
        g = 1.0
        while k > 0.0:
            g *= k
            k -= 1.0
    else:
        k = numpy.ceil(0.5 * dimension)
        g = numpy.sqrt(numpy.pi)
        while k > 0.0:
            g *= k - 0.5
            k -= 1.0
    return g


def ball_radius(volume, dimension):
    return (gamma_function(dimension) * volume) ** (1.0 / dimension) / numpy.sqrt(numpy.pi)


def ball_volume(radius, dimension):
    return (radius * numpy.sqrt(numpy.pi)) ** dimension / gamma_function(dimension)


def kernel_threshold(matrix_size, dimension, density, correlation_scale, nu):
    """_estimate_kernel_threshold :294-413 (with the _ball_volume dimension fix)."""
    adjacency_volume = density * matrix_size
    if adjacency_volume < 1.0:
        raise ValueError('Adjacency: %0.2f. Correlation matrix will become identity '
                         % adjacency_volume)
    gm = numpy.prod(correlation_scale) ** (1.0 / dimension)
    adjacency_volume /= ball_volume(gm, dimension)
    adjacency_radius = ball_radius(adjacency_volume, dimension)
    grid_axis_num_points = matrix_size ** (1.0 / dimension)
    grid_size = 1.0 / (grid_axis_num_points - 1.0)
    kernel_radius = grid_size * adjacency_radius
    return float(matern_kernel(numpy.array([kernel_radius]), nu)[0])


def max_nnz_estimate(matrix_size, correlation_scale, dimension, density):
    """_estimate_max_nnz :420-465 (4-argument form)."""
    est = int(numpy.ceil(density * matrix_size ** 2))
    ncs = correlation_scale / numpy.max(correlation_scale)
    gm = numpy.prod(ncs) ** (1.0 / dimension)
    return int(numpy.ceil(1.0 / ball_radius(gm, dimension) * est))


def sparse_correlation(points, correlation_scale, nu, density, block=1024):
    """CSR of the tapered Matérn matrix: entries with K_ij > threshold."""
    points = numpy.ascontiguousarray(points, dtype=float)
    n, d = points.shape
    scale = broadcast_scale(points, correlation_scale)
    tau = kernel_threshold(n, d, density, scale, nu)
    rows, cols, vals = [], [], []
    for r0 in range(0, n, block):
        r1 = min(n, r0 + block)
        Kb = matern_kernel(scaled_distance(points[r0:r1], points, scale), nu)
        ii, jj = numpy.nonzero(Kb > tau)
        rows.append(ii + r0)
        cols.append(jj)
        vals.append(Kb[ii, jj])
    K = scipy.sparse.csr_matrix((numpy.concatenate(vals),
                                 (numpy.concatenate(rows), numpy.concatenate(cols))),
                                shape=(n, n))
    K.sort_indices()
    return K, tau


# ---------------------------------------------------------------- probes ---

def rademacher_probes(n, num, seed):
    """Counter-based Rademacher probes: bit (i, s) of a splitmix64 hash of
    (seed, s, i) — the same function the device kernel evaluates."""
    i = numpy.arange(n, dtype=numpy.uint64)
    out = numpy.empty((n, num))
    with numpy.errstate(over='ignore'):
        for s in range(num):
            x = (numpy.uint64(seed) * numpy.uint64(0x9E3779B97F4A7C15) +
                 numpy.uint64(s) * numpy.uint64(0xD1B54A32D192ED03) + i)
            x = x + numpy.uint64(0x9E3779B97F4A7C15)
            x = (x ^ (x >> numpy.uint64(30))) * numpy.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> numpy.uint64(27))) * numpy.uint64(0x94D049BB133111EB)
            x = x ^ (x >> numpy.uint64(31))
            out[:, s] = numpy.where((x >> numpy.uint64(63)) == 1, -1.0, 1.0)
    return out


def lanczos(K, v0, steps, reorth=True):
    """Lanczos tridiagonalisation of K from v0 with full reorthogonalisation by
    classical Gram-Schmidt applied twice (CGS2) — the device algorithm.
    Returns (alpha[k], beta[k-1]) with k <= steps (stops on breakdown)."""
    n = v0.shape[0]
    V = numpy.zeros((steps, n))
    alpha, beta = [], []
    v = v0 / numpy.linalg.norm(v0)
    b_prev = 0.0
    v_prev = numpy.zeros(n)
    for k in range(steps):
        V[k] = v
        w = K @ v - b_prev * v_prev
        a = 0.0
        for _ in range(2 if reorth else 1):
            h = V[:k + 1] @ w if reorth else numpy.array([numpy.dot(v, w)])
            w = w - (V[:k + 1].T @ h if reorth else h[0] * v)
            a += h[-1]
        alpha.append(a)
        b = float(numpy.linalg.norm(w))
        if k == steps - 1 or not b > 1e-13 * max(1.0, abs(a)):
            break
        beta.append(b)
        v_prev, v, b_prev = v, w / b, b
    return numpy.array(alpha), numpy.array(beta)


def slq_nodes(alpha, beta):
    """Ritz values theta and weights tau^2 of the Lanczos tridiagonal."""
    T = numpy.diag(alpha) + numpy.diag(beta, 1) + numpy.diag(beta, -1)
    theta, U = numpy.linalg.eigh(T)
    return theta, U[0] ** 2


def slq(K, etas, probes, steps, reorth=True):
    """-> dict(logdet[neta], traceinv[neta], traceinv2[neta]) estimates."""
    n, s = probes.shape
    etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
    ld = numpy.zeros(etas.size)
    t1 = numpy.zeros(etas.size)
    t2 = numpy.zeros(etas.size)
    for p in range(s):
        a, b = lanczos(K, probes[:, p], steps, reorth)
        theta, w = slq_nodes(a, b)
        for e, eta in enumerate(etas):
            ld[e] += numpy.sum(w * numpy.log(theta + eta))
            t1[e] += numpy.sum(w / (theta + eta))
            t2[e] += numpy.sum(w / (theta + eta) ** 2)
    f = n / float(s)
    return dict(logdet=f * ld, traceinv=f * t1, traceinv2=f * t2)
