"""Input generators (oracle restatement; TEST INFRASTRUCTURE ONLY).

Restates /root/reference/examples/_utilities/data_utilities.py:
  generate_points           :22-69   (grid via meshgrid 'xy', x fastest)
  generate_data             :76-129  (sum of sin(pi x_k) + noise, legacy seed 31)
  generate_basis_functions  :136-185 (monomials of total degree <= p)
"""

import numpy


def generate_points(num_points, dimension=2, grid=True, seed=None):
    """data_utilities.py:53-69. ``grid=False`` uses numpy's legacy global RNG
    (reference :67); ``seed`` (our extension) seeds a private RandomState."""
    if grid:
        axis = numpy.linspace(0, 1, num_points)
        mesh = numpy.meshgrid(*([axis] * dimension))        # :56-58, 'xy' indexing
        n = num_points ** dimension
        points = numpy.empty((n, dimension), dtype=float)
        for i in range(dimension):
            points[:, i] = mesh[i].ravel()
        return points
    rng = numpy.random if seed is None else numpy.random.RandomState(seed)
    return rng.rand(num_points, dimension)


def generate_data(points, noise_magnitude):
    """data_utilities.py:92-101: z = sum_k sin(pi x_k) + noise * randn, seed 31."""
    n, d = points.shape
    z = numpy.zeros((n,), dtype=float)
    for i in range(d):
        z += numpy.sin(points[:, i] * numpy.pi)
    rng = numpy.random.RandomState(31)                      # == numpy.random.seed(31)
    z += noise_magnitude * rng.randn(n)
    return z


def generate_basis_functions(points, polynomial_degree=2, trigonometric=False):
    """data_utilities.py:142-185 (same column order as the reference)."""
    n, d = points.shape
    powers_array = numpy.arange(polynomial_degree + 1)
    powers_mesh = numpy.meshgrid(*([powers_array] * d))
    powers_ravel = numpy.array([powers_mesh[i].ravel() for i in range(d)])
    powers = powers_ravel[:, powers_ravel.sum(axis=0) <= polynomial_degree]
    X = numpy.ones((n, powers.shape[1]), dtype=float)
    for j in range(powers.shape[1]):
        for i in range(powers.shape[0]):
            X[:, j] *= points[:, i] ** powers[i, j]
    if trigonometric:                                        # :175-183 (index quirk kept)
        Xt = numpy.empty((n, 2 * d))
        for i in range(d):
            Xt[:, i + 0] = numpy.sin(points[:, i] * numpy.pi)
            Xt[:, i + 1] = numpy.cos(points[:, i] * numpy.pi)
        X = numpy.c_[X, Xt]
    return X
