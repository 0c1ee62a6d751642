"""CPU: the CholeskyQR panel algorithm of the band reduction (shifted
CholeskyQR3 + Householder reconstruction, csrc/gpmi_cholqr.hip) restated in
numpy (tools/cholqr_proto.py), checked as the device kernels rely on it:
H = I - V T V^T is orthogonal, H^T P = [S R; 0] to rounding (also with the
first-order passes), a rank-deficient panel reports failure, and a whole band
reduction with these panels keeps K's spectrum. The GPU tests
(test_gpu_band.py) compare the device panels with the Householder ones."""
import os
import sys

import numpy
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'tools'))
import cholqr_proto as cp  # noqa: E402
from oracle import matern  # noqa: E402


def _check_panel(P, out):
    V, tau, Rhh = out
    m, b = P.shape
    T = cp.t_of(V, tau)
    H = numpy.eye(m) - V @ T @ V.T
    scale = numpy.abs(P).max()
    assert numpy.abs(H.T @ H - numpy.eye(m)).max() < 1e-13
    HtP = H.T @ P
    assert numpy.abs(HtP[b:]).max() < 1e-13 * scale
    assert numpy.abs(HtP[:b] - Rhh).max() < 1e-12 * scale
    assert numpy.all(numpy.triu(Rhh) == Rhh)
    assert numpy.all((tau >= 1.0) & (tau <= 2.0))   # |pivot| + 1 of the signed LU


@pytest.mark.parametrize('cond', [1e2, 1e9, 1e13])
def test_ill_conditioned_panel(cond):
    rng = numpy.random.RandomState(int(numpy.log10(cond)))
    U = numpy.linalg.qr(rng.randn(640, 128))[0]
    W = numpy.linalg.qr(rng.randn(128, 128))[0]
    P = U @ numpy.diag(numpy.logspace(0, -numpy.log10(cond), 128)) @ W
    out, info = cp.cholqr_panel(P)
    assert out is not None, info
    _check_panel(P, out)


def test_first_order_passes_taken_and_exact():
    rng = numpy.random.RandomState(3)
    P = rng.randn(1024, 128)   # well conditioned: passes 2 and 3 are near identity
    out, info = cp.cholqr_panel(P)
    assert info['first_order'], info
    _check_panel(P, out)
    ref, _ = cp.cholqr_panel(P, first_order=False)
    assert numpy.abs(out[2] - ref[2]).max() < 1e-12 * numpy.abs(P).max()


def test_rank_deficient_panel_fails():
    rng = numpy.random.RandomState(4)
    P = rng.randn(512, 100) @ rng.randn(100, 128)   # rank 100
    out, info = cp.cholqr_panel(P)
    assert out is None and 'fail' in info


def test_band_reduction_with_cholqr_panels_keeps_spectrum():
    rng = numpy.random.RandomState(5)
    n = 1152
    K = matern.dense_correlation(rng.rand(n, 2), 0.1, 2.5)
    stats = []
    A = cp.band_reduce_cholqr(K, 128, stats)
    assert all(kind == 'cq' for kind, _ in stats)
    B = numpy.tril(numpy.triu(A, -128), 128)
    lam, lam_ref = numpy.linalg.eigvalsh(B), numpy.linalg.eigvalsh(K)
    assert numpy.abs(lam - lam_ref).max() < 1e-13 * lam_ref.max()
