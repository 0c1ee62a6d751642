from .generate_correlation import generate_correlation, DeviceCorrelation   # noqa: F401
from .generate_correlation import DeviceSparseCorrelation                   # noqa: F401

__all__ = ['generate_correlation']
