"""Matérn correlation matrix generation on the GPU.

Drop-in for ``gaussian_proc.generate_correlation`` of the reference
(gaussian_proc/generate_correlation/generate_correlation.py:32-222): same
signature, same scale broadcast (:190-196), same dense output
(``numpy.ndarray (n, n)``, C order). The pairwise kernel runs on the device
(csrc/gpmi_matern.hip, replacing _generate_dense_correlation.pyx:25-91 and
_kernels.pyx:17-136).

Extension: ``device_resident=True`` returns a :class:`DeviceCorrelation` whose
K never leaves HBM; ``MixedCorrelation`` / ``Likelihood`` / ``GaussianProcess``
accept it in place of the ndarray.
"""

import numpy

from .. import _hip

__all__ = ['generate_correlation', 'DeviceCorrelation', 'DeviceSparseCorrelation']


class DeviceCorrelation(object):
    """A correlation matrix assembled and kept on one GPU."""

    def __init__(self, points, correlation_scale, nu, device=None, max_batch=1):
        self.points = _hip.as_c(points)
        self.correlation_scale = _hip.as_c(correlation_scale)
        self.nu = float(nu)
        n = self.points.shape[0]
        self.shape = (n, n)
        self.op = _hip.Operator(n, device=device, max_batch=max_batch)
        self.op.assemble_matern(self.points, self.correlation_scale, self.nu)

    @property
    def device(self):
        return self.op.device

    def toarray(self):
        """Copy K to the host."""
        return self.op.get_matrix()


class DeviceSparseCorrelation(object):
    """A tapered (compact-support) Matérn correlation kept on one GPU in CSR:
    the entries with matern(x_ij) > tau, tau from the reference's density
    heuristic (``generate_correlation(..., sparse=True)``)."""

    def __init__(self, points, correlation_scale, nu, density, device=None):
        from . import _taper
        self.points = _hip.as_c(points)
        self.correlation_scale = _hip.as_c(correlation_scale)
        self.nu = float(nu)
        self.density = float(density)
        n, d = self.points.shape
        self.shape = (n, n)
        self.tau = _taper.kernel_threshold(n, d, density, self.correlation_scale, nu,
                                           device=device)
        self.op = _hip.SparseOperator.from_points(self.points, self.correlation_scale, self.nu,
                                                  self.tau, device=device)
        self.nnz = self.op.nnz

    @property
    def device(self):
        return self.op.device

    def tocsr(self):
        return self.op.csr()


def _broadcast_scale(points, correlation_scale):
    # generate_correlation.py:191-196
    if numpy.isscalar(correlation_scale):
        return numpy.repeat(numpy.array([correlation_scale], dtype=float), points.shape[1])
    scale = numpy.asarray(correlation_scale, dtype=float).ravel()
    if scale.size != points.shape[1]:
        raise ValueError('correlation_scale must be a scalar or have one entry per '
                         'dimension (%d)' % points.shape[1])
    return scale


def generate_correlation(points, correlation_scale=0.1, nu=0.5, grid=True, sparse=False,
                         density=0.001, plot=False, verbose=False, device=None,
                         device_resident=False, max_batch=1):
    """Matérn correlation matrix of ``points`` (n x d, d <= 8).

    Dense: ``numpy.ndarray`` (n, n). ``sparse=True``: the tapered matrix as a
    ``scipy.sparse.csr_matrix`` (sorted indices), entries with
    matern(x_ij) > tau where tau follows the reference's ``density`` heuristic
    (_generate_sparse_correlation.pyx:294-413, with the argument fixes of
    SURVEY §0.4). ``grid`` and ``plot`` are accepted for signature parity.
    """
    points = numpy.ascontiguousarray(points, dtype=float)
    if points.ndim != 2:
        raise ValueError('points must be a 2D array (num_points, dimension)')
    scale = _broadcast_scale(points, correlation_scale)
    if sparse:
        K = DeviceSparseCorrelation(points, scale, nu, density, device=device)
        if verbose:
            print('Generated sparse correlation matrix of size: %d, nnz: %d, density: %s.'
                  % (points.shape[0], K.nnz, K.nnz / float(points.shape[0]) ** 2))
        return K if device_resident else K.tocsr()
    if device_resident:
        K = DeviceCorrelation(points, scale, nu, device=device, max_batch=max_batch)
    else:
        K = _hip.matern_dense(points, scale, nu, device=device)
    if verbose:
        print('Generated dense correlation matirx of size: %d.' % points.shape[0])
    return K
