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
