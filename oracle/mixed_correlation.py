"""The K + eta*I operator (oracle restatement; TEST INFRASTRUCTURE ONLY).

Restates /root/reference/gaussian_proc/_mixed_correlation/mixed_correlation.py
(``MixedCorrelation`` :25-335) and _linear_solver.py:24-73 for the exact imate
methods ('eigenvalue', 'cholesky'), dense K.
"""

import numpy
import scipy.linalg

from . import imate_exact as imate


class MixedCorrelation(object):
    """mixed_correlation.py:34-79 (dense, interpolate=False)."""

    def __init__(self, K, imate_method='cholesky', imate_options=None):
        self.K = numpy.asarray(K, dtype=float)
        self.imate_method = imate_method
        self.imate_options = dict(imate_options or {})
        self.n = self.K.shape[0]
        self.K_eigenvalues = None
        if imate_method == 'eigenvalue':                    # :76-79
            self.K_eigenvalues = scipy.linalg.eigh(self.K, eigvals_only=True,
                                                   check_finite=False)

    def get_matrix_size(self):                               # :85-90
        return self.n

    def _shifted(self, eta):
        Kn = self.K.copy()
        Kn[numpy.diag_indices(self.n)] += eta
        return Kn

    def trace(self, eta, exponent=1):                        # :96-149
        if exponent == 0:
            t, _ = imate.trace(self.K, exponent=0)
        elif exponent == 1:
            t, _ = imate.trace(self.K, exponent=1)
            if eta != 0:
                t += eta * self.n
        elif exponent == 2:
            if eta == 0:
                t, _ = imate.trace(self.K, exponent=2)
            else:
                tk, _ = imate.trace(self.K, exponent=1)
                tk2, _ = imate.trace(self.K, exponent=2)
                t = tk2 + 2.0 * eta * tk + eta ** 2 * self.n
        elif self.imate_method == 'eigenvalue':
            t, _ = imate.trace(self.K, method='eigenvalue',
                               eigenvalues=self.K_eigenvalues + eta,
                               exponent=exponent)
        else:
            raise ValueError('Existing methods are "exact", "eigenvalue", '
                             'and "slq".')
        return t

    def traceinv(self, eta, exponent=1):                     # :155-215
        if self.imate_method == 'eigenvalue':
            t, _ = imate.traceinv(self.K, method='eigenvalue',
                                  eigenvalues=self.K_eigenvalues + eta,
                                  exponent=exponent)
        elif self.imate_method == 'cholesky':
            t, _ = imate.traceinv(self._shifted(eta), method='cholesky',
                                  exponent=exponent)
        else:
            raise ValueError('Existing methods are "eigenvalue", "cholesky,"'
                             '"hutchinson", and "slq".')
        return t

    def logdet(self, eta, exponent=1):                       # :221-274
        if self.imate_method == 'eigenvalue':
            v, _ = imate.logdet(self.K, method='eigenvalue',
                                eigenvalues=self.K_eigenvalues + eta,
                                exponent=exponent)
        elif self.imate_method in ('cholesky', 'hutchinson'):
            v, _ = imate.logdet(self._shifted(eta), method='cholesky',
                                exponent=exponent)
        else:
            raise ValueError('Existing methods are "eigenvalue", "cholesky",'
                             ' and "slq".')
        return v

    def solve(self, eta, Y):                                 # :280-299 -> _linear_solver.py:71
        return scipy.linalg.solve(self._shifted(eta), Y, assume_a='pos')

    def dot(self, eta, x, exponent=1):                       # :305-335 (p*(K+eta I)x quirk)
        if not isinstance(exponent, int):
            raise ValueError('"exponent" should be an integer.')
        elif exponent < 0:
            raise ValueError('"exponent" should be a non-negative integer.')
        y = numpy.zeros_like(x)
        for _ in range(exponent):
            y += self.K.dot(x)
            if eta != 0:
                y += eta * x
        return y
