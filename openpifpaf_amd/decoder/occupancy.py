"""Occupancy grid (occupancy.py:10-47).  The decoder's own occupancy lives inside the
device grow kernel (csrc/grow.hip); this class keeps the reference API for callers that
use it directly."""
import numpy as np

from ..functional import scalar_nonzero_clipped_with_reduction


def scalar_square_add_single(field, x, y, sigma, value):
    """decoder/utils.py:61-66"""
    minx = max(0, int(x - sigma))
    miny = max(0, int(y - sigma))
    maxx = max(minx + 1, min(field.shape[1], int(x + sigma) + 1))
    maxy = max(miny + 1, min(field.shape[0], int(y + sigma) + 1))
    field[miny:maxy, minx:maxx] += value


class Occupancy():
    def __init__(self, shape, reduction, *, min_scale=None):
        assert len(shape) == 3
        if min_scale is None:
            min_scale = reduction
        assert min_scale >= reduction
        self.reduction = reduction
        self.min_scale = min_scale
        self.min_scale_reduced = min_scale / reduction
        self.occupancy = np.zeros((shape[0], int(shape[1] / reduction),
                                   int(shape[2] / reduction)), dtype=np.uint8)

    def __len__(self):
        return len(self.occupancy)

    def set(self, f, x, y, sigma):
        """Mark a box centred at the rounded (x, y) (u8 += 1, wraps)."""
        if f >= len(self.occupancy):
            return
        xi = round(x / self.reduction)
        yi = round(y / self.reduction)
        si = round(max(self.min_scale_reduced, sigma / self.reduction))
        scalar_square_add_single(self.occupancy[f], xi, yi, si, 1)

    def get(self, f, x, y):
        """Read at the floor of (x, y) / reduction, clipped to the grid."""
        if f >= len(self.occupancy):
            return 1.0
        return scalar_nonzero_clipped_with_reduction(self.occupancy[f], x, y, self.reduction)
