from .gaussian_process import GaussianProcess   # noqa: F401

__all__ = ['GaussianProcess']
