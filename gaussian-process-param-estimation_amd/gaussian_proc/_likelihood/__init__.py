from .likelihood import Likelihood   # noqa: F401

__all__ = ['Likelihood']
