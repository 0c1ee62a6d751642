"""The C-ABI library loads and exports every symbol include/gpmi.h declares
(CPU only: no device calls)."""
import os
import re

import numpy

import pytest

from gaussian_proc import _hip

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      'include', 'gpmi.h')


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*int\s+(gpmi_\w+)\s*\(', src, re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    assert 'gpmi_op_loglik_batch' in syms and 'gpmi_matern_dense' in syms
    assert len(syms) >= 18


def test_library_exports_every_declared_symbol():
    if not os.path.isfile(_hip.LIB_PATH):
        pytest.fail('libgpmi.so missing: run __graft_entry__.build()')
    lib = _hip.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    # and the ctypes binding covers exactly the header
    assert sorted(_hip.SIGNATURES) == declared_symbols()
    assert lib.gpmi_version() >= 100


def test_error_paths_without_device():
    lib = _hip.load()
    # invalid arguments are rejected before any device work
    assert lib.gpmi_op_set_timing(None, 1) < 0
    assert 'null handle' in _hip.last_error()


def test_missing_library_fails_loudly(monkeypatch):
    """No CPU fallback: without libgpmi.so the operator raises ImportError."""
    monkeypatch.setattr(_hip, '_lib', None)
    monkeypatch.setattr(_hip, 'LIB_PATH', '/nonexistent/libgpmi.so')
    with pytest.raises(ImportError):
        _hip.load()
    from gaussian_proc._mixed_correlation import MixedCorrelation
    with pytest.raises(ImportError):
        MixedCorrelation(numpy.eye(4), imate_method='cholesky')


def test_no_device_raises(monkeypatch):
    """On a host without a HIP device the operator raises GPMIError (the CPU
    container), never computes on the host."""
    import torch
    if torch.cuda.is_available():
        pytest.skip('a device is present')
    from gaussian_proc._mixed_correlation import MixedCorrelation
    with pytest.raises(_hip.GPMIError):
        MixedCorrelation(numpy.eye(4), imate_method='cholesky')
