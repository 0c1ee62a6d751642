"""The bench's own inputs are pinned: gaussian_proc._data (the product-side
generator bench.py feeds the timed run) equals the oracle restatement of
examples/_utilities/data_utilities.py:22-185 bit for bit, and both reproduce the
reference's own arrays / sums recorded in tests/golden (make_golden.py ran the
reference's data_utilities)."""

import numpy
import pytest

from gaussian_proc import _data
from oracle import data
from _util import load_json, load_npz

# (points per axis, dimension): cfg1, cfg2, n1024, cfg3, cfg4, cfg5
SIZES = [(256, 1), (64, 2), (32, 2), (128, 2), (256, 2), (64, 3)]


@pytest.mark.parametrize('npts,d', SIZES)
def test_product_generators_equal_oracle_bitwise(npts, d):
    p1 = _data.generate_points(npts, d, True)
    p2 = data.generate_points(npts, d, True)
    numpy.testing.assert_array_equal(p1, p2)
    numpy.testing.assert_array_equal(_data.generate_data(p1, 0.2), data.generate_data(p2, 0.2))
    numpy.testing.assert_array_equal(_data.generate_basis_functions(p1, 2),
                                     data.generate_basis_functions(p2, 2))
    # the trigonometric columns the reference writes (its index quirk leaves the
    # last one unset; numpy.empty in both)
    X1 = _data.generate_basis_functions(p1, 2, trigonometric=True)
    X2 = data.generate_basis_functions(p2, 2, trigonometric=True)
    m = X1.shape[1] - 2 * d
    numpy.testing.assert_array_equal(X1[:, :m + d + 1], X2[:, :m + d + 1])


def test_product_generators_equal_reference_arrays_cfg1():
    arr = load_npz('cfg1_arrays.npz')
    pts = _data.generate_points(256, 1, True)
    numpy.testing.assert_array_equal(pts, arr['points'])
    numpy.testing.assert_array_equal(_data.generate_data(pts, 0.2), arr['z'])
    numpy.testing.assert_array_equal(_data.generate_basis_functions(pts, 2), arr['X'])


@pytest.mark.parametrize('fixture,npts,d', [('cfg1.json', 256, 1), ('cfg2.json', 64, 2),
                                            ('n1024_nu25.json', 32, 2)])
def test_product_generators_match_reference_sums(fixture, npts, d):
    g = load_json(fixture)
    pts = _data.generate_points(npts, d, True)
    z = _data.generate_data(pts, 0.2)
    X = _data.generate_basis_functions(pts, 2)
    assert (g['n'], g['m']) == X.shape
    assert float(z.sum()) == g['z_sum']
    numpy.testing.assert_array_equal(z[g['sample_rows']], g['z_samples'])
    numpy.testing.assert_array_equal(X.sum(axis=0), g['X_col_sums'])
