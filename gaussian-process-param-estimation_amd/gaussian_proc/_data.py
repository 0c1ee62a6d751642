"""Synthetic inputs of the reference's benchmarks (product-side utility).

Same definitions as the reference's examples/_utilities/data_utilities.py
(generate_points :22-69, generate_data :76-129 with numpy's legacy seed 31,
generate_basis_functions :136-185), used by bench.py and the examples.
"""

import numpy

__all__ = ['generate_points', 'generate_data', 'generate_basis_functions']


def generate_points(num_points, dimension=2, grid=True):
    if not grid:
        return numpy.random.rand(num_points, dimension)
    axis = numpy.linspace(0.0, 1.0, num_points)
    mesh = numpy.meshgrid(*([axis] * dimension))
    return numpy.stack([m.ravel() for m in mesh], axis=1).astype(float)


def generate_data(points, noise_magnitude):
    # accumulate in the reference order (dimension by dimension)
    z = numpy.zeros(points.shape[0])
    for k in range(points.shape[1]):
        z += numpy.sin(points[:, k] * numpy.pi)
    return z + noise_magnitude * numpy.random.RandomState(31).randn(points.shape[0])


def generate_basis_functions(points, polynomial_degree=2, trigonometric=False):
    n, d = points.shape
    grids = numpy.meshgrid(*([numpy.arange(polynomial_degree + 1)] * d))
    powers = numpy.array([g.ravel() for g in grids])
    powers = powers[:, powers.sum(axis=0) <= polynomial_degree]
    X = numpy.ones((points.shape[0], powers.shape[1]))
    for j in range(powers.shape[1]):
        for i in range(d):
            X[:, j] *= points[:, i] ** powers[i, j]
    if trigonometric:
        # reference :175-183, its column index quirk included (i + 0 / i + 1
        # overlap for d > 1, so sin of axis i is overwritten by cos of axis i - 1)
        T = numpy.empty((n, 2 * d))
        for i in range(d):
            T[:, i] = numpy.sin(points[:, i] * numpy.pi)
            T[:, i + 1] = numpy.cos(points[:, i] * numpy.pi)
        X = numpy.c_[X, T]
    return X
