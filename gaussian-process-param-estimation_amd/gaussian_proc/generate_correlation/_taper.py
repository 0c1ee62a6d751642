"""Taper threshold of the sparse (compact-support) Matérn correlation.

Restates the reference heuristic of
gaussian_proc/generate_correlation/_generate_sparse_correlation.pyx with the two
argument fixes of SURVEY §0.4 (the shipped file raises TypeError):
  gamma_function :208-233, _ball_radius / _ball_volume :240-287,
  _estimate_kernel_threshold :294-413 (``_ball_volume(r)`` -> ``_ball_volume(r, d)``).
The final kernel value is evaluated by the same device Matérn kernel that
assembles the matrix, so the kept set is consistent with the device entries.
"""

import numpy

from .. import _hip


def _gamma_half(dimension):
    """Gamma(dimension / 2 + 1) by the reference's product recurrences."""
    if dimension % 2 == 0:
        k, g = 0.5 * dimension, 1.0
        while k > 0.0:
            g *= k
            k -= 1.0
        return g
    k, g = numpy.ceil(0.5 * dimension), numpy.sqrt(numpy.pi)
    while k > 0.0:
        g *= k - 0.5
        k -= 1.0
    return g


def _ball_radius(volume, dimension):
    return (_gamma_half(dimension) * volume) ** (1.0 / dimension) / numpy.sqrt(numpy.pi)


def _ball_volume(radius, dimension):
    return (radius * numpy.sqrt(numpy.pi)) ** dimension / _gamma_half(dimension)


def taper_radius(matrix_size, dimension, density, correlation_scale):
    """Scaled kernel radius whose Matérn value is the taper threshold."""
    adjacency = density * matrix_size
    if adjacency < 1.0:
        raise ValueError(
            'Adjacency: %0.2f. Correlation matrix will become identity ' % adjacency +
            'since kernel radius is less than grid size. To increase ' +
            'adjacency, consider increasing density or correlation_scale.')
    gm = numpy.prod(correlation_scale) ** (1.0 / dimension)
    adjacency /= _ball_volume(gm, dimension)
    radius = _ball_radius(adjacency, dimension)
    grid_size = 1.0 / (matrix_size ** (1.0 / dimension) - 1.0)
    return grid_size * radius


def kernel_threshold(matrix_size, dimension, density, correlation_scale, nu, device=None):
    r = taper_radius(matrix_size, dimension, density, correlation_scale)
    return float(_hip.matern_values([r], nu, device=device)[0])
