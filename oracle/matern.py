"""Matérn correlation assembly (oracle restatement; TEST INFRASTRUCTURE ONLY).

Restates
  matern_kernel               generate_correlation/_kernels.pyx:17-100
  euclidean_distance          generate_correlation/_kernels.pyx:107-136
  _generate_correlation_matrix generate_correlation/_generate_dense_correlation.pyx:25-91
  generate_correlation (scale broadcast)  generate_correlation.py:190-196
"""

import numpy
import scipy.special


def matern_kernel(x, nu):
    """Vectorised _kernels.pyx:73-93. x==0 -> 1; closed forms for nu in
    {0.5, 1.5, 2.5}; 2^(1-nu)/Gamma(nu) (sqrt(2nu)x)^nu K_nu(sqrt(2nu)x) for
    nu < 100; Gaussian exp(-x^2/2) otherwise."""
    x = numpy.asarray(x, dtype=float)
    out = numpy.ones_like(x)
    nz = x != 0
    xs = x[nz]
    if nu == 0.5:
        v = numpy.exp(-xs)
    elif nu == 1.5:
        s3 = numpy.sqrt(3.0)
        v = (1.0 + s3 * xs) * numpy.exp(-s3 * xs)
    elif nu == 2.5:
        s5 = numpy.sqrt(5.0)
        v = (1.0 + s5 * xs + (5.0 / 3.0) * (xs ** 2)) * numpy.exp(-s5 * xs)
    elif nu < 100:
        t = numpy.sqrt(2.0 * nu) * xs
        v = ((2.0 ** (1.0 - nu)) / scipy.special.gamma(nu)) * (t ** nu) * \
            scipy.special.kv(nu, t)
    else:
        v = numpy.exp(-0.5 * xs ** 2)
    out[nz] = v
    return out


def scaled_distance(p1, p2, scale):
    """_kernels.pyx:130-136: sqrt(sum_k ((p1_k - p2_k)/rho_k)^2), summed in k order.
    p1: [a, d], p2: [b, d] -> [a, b]."""
    d = p1.shape[1]
    acc = numpy.zeros((p1.shape[0], p2.shape[0]))
    for k in range(d):
        acc += ((p1[:, k][:, None] - p2[:, k][None, :]) / scale[k]) ** 2
    return numpy.sqrt(acc)


def broadcast_scale(points, correlation_scale):
    """generate_correlation.py:191-196."""
    if numpy.isscalar(correlation_scale):
        return numpy.repeat(numpy.array([correlation_scale], dtype=float),
                            points.shape[1])
    return numpy.asarray(correlation_scale, dtype=float)


def dense_correlation(points, correlation_scale=0.1, nu=0.5, block=2048):
    """Dense K (n x n, C order), _generate_dense_correlation.pyx:77-91.
    The reference evaluates the upper triangle and mirrors it; the kernel is
    symmetric in (i, j) bit-for-bit, so evaluating every pair is equivalent."""
    points = numpy.ascontiguousarray(points, dtype=float)
    scale = broadcast_scale(points, correlation_scale)
    n = points.shape[0]
    K = numpy.empty((n, n))
    for r0 in range(0, n, block):
        r1 = min(n, r0 + block)
        K[r0:r1] = matern_kernel(scaled_distance(points[r0:r1], points, scale), nu)
    return K
