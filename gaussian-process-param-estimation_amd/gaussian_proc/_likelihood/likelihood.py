"""Likelihood facade (drop-in for gaussian_proc/_likelihood/likelihood.py:23-102).

The reference builds ``MixedCorrelation(K, interpolate=False,
imate_method='eigenvalue')`` (:40-49): a one-time dense eigh, then 2 dense
solves per evaluation. Here the same 'eigenvalue' operator is device-resident:
its one-time setup is the band reduction K = Q B Q^T (bandwidth 128), after
which every evaluation is one banded Cholesky of B + eta I (exact, same values
to rounding); traceinv / trace use the device eigenvalues of B. ``max_batch``
sizes the dense per-eta Cholesky workspace the operator's 'cholesky' calls
(solve, hutchinson) use.
"""

from .._mixed_correlation import MixedCorrelation
from ._direct_likelihood import DirectLikelihood
from ._profile_likelihood import ProfileLikelihood

__all__ = ['Likelihood']


class Likelihood(object):

    def __init__(self, X, K, likelihood_method='direct', device=None, max_batch=None):
        self.X = X
        self.K = K
        self.likelihood_method = likelihood_method
        self.K_mixed = MixedCorrelation(K, interpolate=False, imate_method='eigenvalue',
                                        imate_options={}, device=device,
                                        max_batch=max_batch)

    def likelihood(self, z, hyperparam):                       # :55-61
        return DirectLikelihood.log_likelihood(z, self.X, self.K_mixed, False, hyperparam)

    def likelihood_batch(self, z, hyperparams):
        """log-likelihood at many (sigma, sigma0) pairs (batched device calls)."""
        return DirectLikelihood.log_likelihood_batch(z, self.X, self.K_mixed, hyperparams)

    def maximize_log_likelihood(self, z, plot=False):          # :67-102
        if self.likelihood_method == 'direct':
            results = DirectLikelihood.maximize_log_likelihood(z, self.X, self.K_mixed)
        elif self.likelihood_method == 'profiled':
            interval_eta = [1e-4, 1e+3]                         # :90
            results = ProfileLikelihood.find_log_likelihood_der1_zeros(
                z, self.X, self.K_mixed, interval_eta)
        else:
            raise ValueError('likelihood_method must be "direct" or "profiled".')
        if plot:
            print('plotting is not part of the device build; skipped')
        return results
