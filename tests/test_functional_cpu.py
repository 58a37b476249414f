"""The host twins of the functional primitives (pp_*_cpu, openpifpaf_amd.functional_cpu)
against the reference's known-answer vectors (tests/golden/primitives.npz, produced by the
reference's functional.pyx), bit-exact -- the same vectors the device kernels are checked
against in test_gpu_parity.py.  Runs without a GPU: these entry points take host pointers.
"""
import numpy as np
import pytest

import golden_util as gu
from openpifpaf_amd import functional_cpu as F


@pytest.fixture(scope='module')
def prim():
    return gu.load_primitives()


def _pts(p, key):
    return [np.ascontiguousarray(r) for r in p[key]]


@pytest.mark.parametrize('t', range(4))
def test_add_gauss_with_max(prim, t):
    field = prim['sqg_max_%d_in' % t].copy()
    trunc, maxv = prim['sqg_max_%d_args' % t]
    F.scalar_square_add_gauss_with_max(field, *_pts(prim, 'sqg_max_%d_pts' % t),
                                       truncate=trunc, max_value=maxv)
    assert np.array_equal(field, prim['sqg_max_%d_out' % t])


def test_add_gauss_with_max_strided_and_empty(prim):
    big = prim['sqg_max_strided_in'].copy()
    F.scalar_square_add_gauss_with_max(big[::2, 1::2], *_pts(prim, 'sqg_max_strided_pts'),
                                       truncate=1.0)
    assert np.array_equal(big, prim['sqg_max_strided_out'])
    field = prim['sqg_max_empty_in'].copy()
    e = np.zeros(0, np.float32)
    F.scalar_square_add_gauss_with_max(field, e, e, e, e)
    assert np.array_equal(field, prim['sqg_max_empty_out'])


@pytest.mark.parametrize('t', range(2))
def test_add_gauss(prim, t):
    field = prim['sqg_%d_in' % t].copy()
    F.scalar_square_add_gauss(field, *_pts(prim, 'sqg_%d_pts' % t),
                              truncate=prim['sqg_%d_args' % t][0])
    assert np.array_equal(field, prim['sqg_%d_out' % t])


@pytest.mark.parametrize('t', range(2))
def test_max_gauss(prim, t):
    field = prim['sqmax_%d_in' % t].copy()
    F.scalar_square_max_gauss(field, *_pts(prim, 'sqmax_%d_pts' % t),
                              truncate=prim['sqmax_%d_args' % t][0])
    assert np.array_equal(field, prim['sqmax_%d_out' % t])


def test_add_constant(prim):
    field = prim['sqc_in'].copy()
    F.scalar_square_add_constant(field, *_pts(prim, 'sqc_pts'))
    assert np.array_equal(field, prim['sqc_out'])


def test_cumulative_average(prim):
    cuma, cumw = [a.copy() for a in prim['cuma_in']]
    F.cumulative_average(cuma, cumw, *_pts(prim, 'cuma_pts'))
    assert np.array_equal(np.stack([cuma, cumw]), prim['cuma_out'])


@pytest.mark.parametrize('t', range(3))
def test_weiszfeld(prim, t):
    y = prim['weisz_%d_y0' % t].copy()
    y_out, denom = F.weiszfeld_nd(prim['weisz_%d_x' % t], y, prim['weisz_%d_w' % t])
    assert y_out is y
    assert np.array_equal(y, prim['weisz_%d_y' % t])
    assert np.array_equal(denom, prim['weisz_%d_denom' % t])


def test_lookups(prim):
    f = prim['lookup_field']
    px, py = prim['lookup_pts']
    assert np.array_equal(F.scalar_values(f, px, py), prim['scalar_values'])
    assert np.array_equal(F.scalar_values(f, px, py, 0.0), prim['scalar_values_d0'])
    occ = prim['lookup_occ']
    got = [[F.scalar_value(f, x, y, -1.0), F.scalar_value_clipped(f, x, y),
            F.scalar_nonzero(occ, x, y, 0), F.scalar_nonzero_clipped(occ, x, y),
            F.scalar_nonzero_clipped_with_reduction(occ, 2 * x, 2 * y, 2.0)]
           for x, y in zip(px, py)]
    got = np.array(got)
    for col, key in enumerate(('scalar_value', 'scalar_value_clipped', 'scalar_nonzero',
                               'scalar_nonzero_clipped', 'scalar_nonzero_red')):
        assert np.array_equal(got[:, col].astype(prim[key].dtype), prim[key]), key


def test_center_filters(prim):
    caf = prim['center_field']
    for t, (qx, qy, qs) in enumerate(prim['center_queries']):
        assert np.array_equal(F.caf_center_s(caf, qx, qy, qs), prim['caf_center_s_%d' % t])
        assert np.array_equal(F.paf_center(caf[:7], qx, qy, qs), prim['paf_center_%d' % t])
        assert np.array_equal(F.paf_center_b(caf[:7], qx, qy, np.float32(qs / 3)),
                              prim['paf_center_b_%d' % t])
        assert np.array_equal(F.paf_mask_center(caf[:7], qx, qy, np.float32(qs / 3)),
                              prim['paf_mask_center_%d' % t])


def test_occupancy_set_matches_reference_restatement():
    """Occupancy.set (occupancy.py:36-44 + utils.py:61-66) restated on a NumPy grid: f32
    division, half-to-even rounding, the u8 wrap, marks on planes past the grid skipped."""
    rng = np.random.default_rng(3)
    grid = np.zeros((5, 18, 14), np.uint8)
    ref = grid.copy()
    marks = [(int(rng.integers(0, 6)), np.float32(rng.uniform(-5, 40)),
              np.float32(rng.uniform(-5, 45)), np.float32(rng.uniform(0, 12)))
             for _ in range(200)]
    marks += [(1, np.float32(9.0), np.float32(11.0), np.float32(1.0))] * 260  # wraps past 255
    for f, x, y, s in marks:
        if f >= len(ref):
            continue
        xi, yi = round(x / np.float32(2)), round(y / np.float32(2))
        si = round(max(np.float32(2.0), s / np.float32(2)))
        minx, miny = max(0, int(xi - si)), max(0, int(yi - si))
        maxx = max(minx + 1, min(ref.shape[2], int(xi + si) + 1))
        maxy = max(miny + 1, min(ref.shape[1], int(yi + si) + 1))
        ref[f][miny:maxy, minx:maxx] += np.uint8(1)
    F.occupancy_set(grid, [m[0] for m in marks], [m[1] for m in marks], [m[2] for m in marks],
                    [m[3] for m in marks], 2.0, 2.0)
    assert np.array_equal(grid, ref)


def test_admission_errors_match_device_api():
    """The reference's typed-memoryview ValueErrors (errors.json), as the device API raises
    them, and device tensors refused."""
    errs = gu.load_errors()
    field = np.zeros((4, 4), np.float64)
    pts = [np.zeros(1, np.float32)] * 4
    with pytest.raises(ValueError) as e:
        F.scalar_square_add_gauss_with_max(field, *pts)
    assert ['ValueError', str(e.value)] in list(errs.values())
    with pytest.raises(ValueError, match='wrong number of dimensions'):
        F.scalar_values(np.zeros(4, np.float32), pts[0], pts[1])
    import torch
    with pytest.raises(TypeError):
        F.scalar_values(torch.zeros((4, 4)), pts[0], pts[1])
