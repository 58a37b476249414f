"""Network-output ingestion on the device (network/heads.py).

`fields_from_conv` turns the raw conv output of a CompositeFieldFused head into the
decoder's fields in one HIP pass (pp_fields_from_conv): the eval-mode tail of
CompositeFieldFused.forward (heads.py:406-455) and CifCafCollector / CifdetCollector
(heads.py:65-88, 127-144) fused.  `CifCafCollector` keeps the reference collector's role
for a model whose heads stop at their conv: forward(conv outputs) -> (cif, caf).
"""
import torch

from . import _device
from ._lib import call, load

LAYOUTS = {'cif': (0, 5), 'caf': (1, 9), 'cifdet': (2, 7)}


def fields_dim(n, quad):
    """Field size after `quad` PixelShuffle(2) dequads with the last row / column dropped."""
    return int(load().pp_fields_dim(int(n), int(quad)))


def fields_from_conv(conv, n_fields, kind, quad=1):
    """conv (B, n_fields * per_field * 4^quad, h, w) float32 device tensor -> decoder
    fields (B, n_fields, 5 | 9 | 7, H, W) for kind 'cif' | 'caf' | 'cifdet'."""
    layout, n_out = LAYOUTS[kind]
    conv = _device.to_device(conv)
    b, ch, h, w = conv.shape
    if ch != n_fields * n_out * 4 ** quad:
        raise ValueError('{} conv expects {} channels, got {}'.format(
            kind, n_fields * n_out * 4 ** quad, ch))
    out = torch.empty((b, n_fields, n_out, fields_dim(h, quad), fields_dim(w, quad)),
                      dtype=torch.float32, device=conv.device)
    call('pp_fields_from_conv', _device.ptr(conv), b, n_fields, layout, h, w, quad,
         _device.ptr(out), _device.stream())
    return out


class CifCafCollector(torch.nn.Module):
    """heads.CifCafCollector for heads that stop at their conv: forward((cif_conv,
    caf_conv)) -> (cif, caf) in the decoder layout, on the device."""

    def __init__(self, n_cif, n_caf, quad=1):
        super().__init__()
        self.n_cif, self.n_caf, self.quad = n_cif, n_caf, quad

    def forward(self, *args):  # pylint: disable=arguments-differ
        cif_conv, caf_conv = args[0]
        return (fields_from_conv(cif_conv, self.n_cif, 'cif', self.quad),
                fields_from_conv(caf_conv, self.n_caf, 'caf', self.quad))


class CifdetCollector(torch.nn.Module):
    """heads.CifdetCollector for a detection head that stops at its conv."""

    def __init__(self, n_categories, quad=1):
        super().__init__()
        self.n_categories, self.quad = n_categories, quad

    def forward(self, *args):  # pylint: disable=arguments-differ
        return (fields_from_conv(args[0][0], self.n_categories, 'cifdet', self.quad),)
