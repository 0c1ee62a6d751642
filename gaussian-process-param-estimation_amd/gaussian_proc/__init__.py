"""gaussian_proc — MI355X-native (gfx950 HIP) drop-in for the hot path of
ameli/gaussian-process-param-estimation v0.0.1.

Same public names as the reference (gaussian_proc/__init__.py:72-77):
``GaussianProcess`` and ``generate_correlation``; the likelihood and operator
layers (``gaussian_proc._likelihood.Likelihood``,
``gaussian_proc._mixed_correlation.MixedCorrelation``) keep the reference
signatures. All numerics run through libgpmi.so (include/gpmi.h); there is no
CPU fallback.
"""

from .generate_correlation import generate_correlation, DeviceCorrelation   # noqa: F401
from .gaussian_process import GaussianProcess                              # noqa: F401
from .__version__ import __version__                                       # noqa: F401

__all__ = ['GaussianProcess', 'generate_correlation']
