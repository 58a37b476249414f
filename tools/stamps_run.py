"""Diagnostic: run the decode with the stamps build and print per-section cycle shares.

    PP_LIB_VARIANT=stamps PP_STAMPS_OUT=gpurun_out/stamps.bin python tools/stamps_run.py \
        [kind:n:side[:dense] ...]   (default planted:256:80 uniform:32:80; dense = the
        44-CAF DENSE_DECODE_SKELETON of cfg5)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, make_config  # noqa: E402
from openpifpaf_amd.engine import DecodeEngine  # noqa: E402

P1 = ['seed_scan', 'plan', 'round_grow', 'commit+mark', 'cache_commit', 'helper grow cyc']
# (seed_loop_kernel: slot 5 = the helpers' grow cycles, slot 8 = their grow count)
# phase 1 slots 6 / 7: rounds (grows on wave 0) and annotations taken from the cache
P2 = ['load', 'complete']  # summed over the image's kCompleteWays workgroups
P3 = ['load', '-', 'nms_filter', 'nms_sort', 'nms_occ', 'nms_clear', 'nms_refilter',
      'nms_sort2', 'output']

out = os.environ.get('PP_STAMPS_OUT', 'pp_stamps.bin')
cases = sys.argv[1:] or ['planted:256:80', 'uniform:32:80']
for case in cases:
    kind, n, h = case.split(':')[:3]
    n, h = int(n), int(h)
    dense = case.endswith(':dense')
    skel = constants.DENSE_DECODE_SKELETON if dense else constants.COCO_PERSON_SKELETON
    kw = {}
    if dense:
        kw = {'n_caf': len(skel)} if kind == 'uniform' else {'skeleton': skel, 'n_people': 16}
    if os.path.exists(out):
        os.remove(out)
    cif, caf = synthetic.batch(kind, n, h, h, **kw)
    eng = DecodeEngine()
    cfg = make_config(**EVAL_CONFIG)
    c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
    for _ in range(2):
        b = eng.launch(c, f, skel, cfg)
    torch.cuda.synchronize()
    n_ann = b.counts.cpu().numpy()
    n_seed_cells = (cif[:, :, 0] > cfg.seed_threshold).reshape(n, -1).sum(axis=1)
    st = np.fromfile(out, dtype=np.uint64).reshape(-1, n, 3, 16)[-1].astype(np.float64)
    print('== {} (mean shader cycles per image)'.format(case))
    for ph, names in ((0, P1), (1, P2), (2, P3)):
        tot = st[:, ph, :min(len(names), 5 if ph == 0 else 8)].sum(axis=1).mean()
        print('  phase {} total {:.3e}'.format(ph + 1, tot))
        for i, name in enumerate(names):
            m = st[:, ph, i].mean()
            print('    {:14s} {:12.0f}  {:5.1f}%'.format(name, m, 100 * m / max(tot, 1)))
        if ph == 0:
            print('    rounds {:.1f}  cache hits {:.1f}'.format(st[:, 0, 6].mean(), st[:, 0, 7].mean()))
            per = st[:, 0, :5].sum(axis=1)
            w = int(np.argmax(per))
            print('    per-image total: p50 {:.3e} p90 {:.3e} max {:.3e} (image {}: rounds {:.0f}, '
                  'hits {:.0f}, round_grow {:.3e})'.format(
                      np.percentile(per, 50), np.percentile(per, 90), per[w], w, st[w, 0, 6],
                      st[w, 0, 7], st[w, 0, 2]))
            top = np.argsort(-per)[:8]
            print('    heaviest images (cycles, rounds, hits, anns, seed cells):')
            for t in top:
                print('      {:4d} {:.3e} {:3.0f} {:3.0f} {:4d} {:5d}'.format(
                    t, per[t], st[t, 0, 6], st[t, 0, 7], n_ann[t], n_seed_cells[t]))
            print('    corr(cycles, anns) {:.2f}  corr(cycles, rounds) {:.2f}  corr(cycles, seed cells) {:.2f}'.format(
                np.corrcoef(per, n_ann)[0, 1], np.corrcoef(per, st[:, 0, 6])[0, 1],
                np.corrcoef(per, n_seed_cells)[0, 1]))
        if ph == 0 and st[:, 0, 5].mean() > 0:  # seed_loop_kernel: the helpers' plans, wave 0's waits
            w15 = np.fromfile(out, dtype=np.uint64).reshape(-1, n, 3, 16)[-1][:, 0, 15]
            print('    [one-CU kernel] helper plan cyc {:.0f}  self plans {:.1f}  wave 0 hit wait {:.0f}'.format(
                st[:, 0, 14].mean(), (w15 >> np.uint64(40)).astype(np.float64).mean(),
                (w15 & np.uint64((1 << 40) - 1)).astype(np.float64).mean()))
        for i, name in ((8, 'n connection' if ph else 'helper grows'), (9, 'in-grow pop'), (10, 'in-grow connection'),
                        (11, 'in-grow add'), (12, ' eval: loads / ext plan: filter+picks'),
                        (13, ' eval: forward / ext hit: wait'),
                        (14, ' plan: ext refresh' if ph == 0 else '-'),
                        (15, ' plan: ext CAS' if ph == 0 else '-')):
            print('    {:14s} {:12.0f}'.format(name, st[:, ph, i].mean()))
