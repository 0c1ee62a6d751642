from .mixed_correlation import MixedCorrelation   # noqa: F401

__all__ = ['MixedCorrelation']
