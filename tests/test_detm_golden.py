"""CPU checks of the multi-head CifDet fixtures (tests/golden/detm_*.npz, made by
gen_golden.gen_det_multi from the reference): the per-head inputs regenerate bit for bit from
their recorded generator parameters, and the recorded outputs are consistent with the
reference's orders (get() = sorted(seeds, reverse=True); fields of known categories).  The
decoder itself is compared with them on the GPU (test_gpu_parity.py::test_cifdet_multi_*)."""
import glob
import os

import numpy as np
import pytest

import golden_util as gu

NAMES = sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(gu.GOLDEN, 'detm_*.npz')))


def test_fixtures_present():
    assert {'m2_p', 'm2_pms', 'm1_ums'} <= set(NAMES)


@pytest.mark.parametrize('name', NAMES)
def test_detm_inputs_and_orders(name):
    from openpifpaf_amd import synthetic
    g = np.load(os.path.join(gu.GOLDEN, 'detm_%s.npz' % name))
    k = int(g['n_categories'])
    for (h, w, stride, ms, seed), want in zip(g['heads'], g['input_sha']):
        f = synthetic.det_batch(str(g['gen']), 1, int(h), int(w), first_seed=int(seed),
                                n_categories=k)[0]
        assert gu.sha(f) == str(want)
    seeds = [tuple(r) for r in g['seeds'].tolist()]
    assert seeds == sorted(seeds, reverse=True)
    assert ((g['ann_field'] >= 0) & (g['ann_field'] < k)).all()
    assert len(g['ann_score']) == len(g['ann_bbox'])
    if any(ms for _, _, _, ms, _ in g['heads']):  # the min-scale cases do filter seeds
        assert len(seeds) > 0
