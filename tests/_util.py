"""Shared helpers for the test-suite (fixtures loading, config inputs)."""
import json
import os

import numpy

from oracle import data

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def load_npz(name):
    return numpy.load(os.path.join(GOLDEN, name), allow_pickle=False)


def config_inputs(cfg):
    """points, z, X of a golden config (data_utilities.py restated in oracle.data)."""
    pts = data.generate_points(cfg['num_points'], cfg['dimension'], True)
    z = data.generate_data(pts, 0.2)
    X = data.generate_basis_functions(pts, 2)
    return pts, z, X


def rel(a, b):
    a = numpy.asarray(a, dtype=float)
    b = numpy.asarray(b, dtype=float)
    return numpy.max(numpy.abs(a - b) / numpy.maximum(numpy.abs(b), 1e-300))


def check_der1_sequence(memo, seq, n_exact=3):
    """The (log10 eta, der1) points the reference's profiled driver evaluated
    (seq, recorded by make_golden.py) against the memo of ours: the bracket
    search and the first Chandrupatla point (the first n_exact) are the same
    floats; later interpolation points depend on der1 values that, near the
    root, are dominated by rounding (cancellation), so there only the points
    that coincide are compared by value."""
    keys = numpy.array(sorted(memo))
    scale = max(abs(v) for _, v in seq)
    for i, (le, v) in enumerate(seq):
        k = keys[numpy.argmin(numpy.abs(keys - le))]
        if i < n_exact:
            assert k == le, (i, le, k)
        elif abs(k - le) > 1e-12 * max(1.0, abs(le)):
            continue
        assert abs(memo[k] - v) <= 1e-9 * scale + 1e-6 * abs(v), (le, memo[k], v)
