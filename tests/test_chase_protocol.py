"""CPU check of the systolic bulge-chase protocols the device kernels implement
(csrc/gpmi_chase.hip: chase_systolic_kernel, chase_split_kernel): the numpy
restatement in tools/chase_systolic_proto.py keeps each chase position's blocks in
circular (physical = logical + sweep) layout, exchanges only the messages the
kernels exchange, and slides its windows the same way. Its tridiagonal must have
the band matrix's spectrum (1e-13 relative) at ragged sizes, including n < b and
the last position's partial blocks."""

import importlib.util
import os

import numpy
import pytest

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools',
                     'chase_systolic_proto.py')
_spec = importlib.util.spec_from_file_location('chase_systolic_proto', _PATH)
proto = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(proto)


def _band(n, b, seed):
    rng = numpy.random.RandomState(seed)
    X = rng.randn(n, n)
    S = X + X.T
    i = numpy.arange(n)
    return numpy.where(numpy.abs(numpy.subtract.outer(i, i)) <= b, S, 0.0)


def _tridiag_eigs(d, e2):
    e = numpy.sqrt(e2[:-1])
    return numpy.linalg.eigvalsh(numpy.diag(d) + numpy.diag(e, 1) + numpy.diag(e, -1))


@pytest.mark.parametrize('n,b', [(3, 4), (9, 4), (37, 4), (64, 8), (129, 8), (130, 16)])
@pytest.mark.parametrize('form', ['chase', 'chase_split'])
def test_systolic_protocol_preserves_spectrum(n, b, form):
    Bm = _band(n, b, n + b)
    d, e2 = getattr(proto, form)(numpy.tril(Bm), b)
    ref = numpy.linalg.eigvalsh(Bm)
    assert numpy.max(numpy.abs(_tridiag_eigs(d, e2) - ref)) <= 1e-13 * numpy.abs(ref).max()
