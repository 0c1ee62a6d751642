"""Gaussian process user class (drop-in for
gaussian_proc/gaussian_process/gaussian_process.py:21-71)."""

from .._likelihood import Likelihood

__all__ = ['GaussianProcess']


class GaussianProcess(object):
    """Gaussian process for regression with basis X (n x m) and correlation K
    (n x n ndarray, or a DeviceCorrelation from
    ``generate_correlation(..., device_resident=True)``)."""

    def __init__(self, X, K, likelihood_method='direct', device=None):
        self.X = X
        self.K = K
        self.likelihood = Likelihood(X, K, likelihood_method=likelihood_method,
                                     device=device)

    def train(self, z, plot=False):
        """Find the hyperparameters; prints the results dict (reference :154-162)."""
        results = self.likelihood.maximize_log_likelihood(z, plot=plot)
        print(results)
