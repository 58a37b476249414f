"""Reference decoder vs oracle on this container's CPU (THIS CONTAINER ONLY: imports the
reference from /root/reference through oracle/ref_loader.py).

    python tools/cpu_ratio.py      -> profiles/cpu_ratio.json

The reference's Cython decoder cannot travel to the GPU box, so bench.py's cpu_baseline
times the oracle (oracle/pp_oracle.c) there.  This script times both on the same images,
one thread, median per image, so the bench line can state the reference-equivalent
number: reference images/s = oracle images/s / ratio.
"""
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'oracle'))
sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))

import oracle  # noqa: E402
import ref_loader  # noqa: E402
from gen_golden import configure  # noqa: E402
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, make_config  # noqa: E402


def med_ms(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts))


def main():
    op = ref_loader.load()
    dec = op.decoder
    configure(dec, 'eval', {})
    cfg = make_config(**EVAL_CONFIG)
    skel = constants.COCO_PERSON_SKELETON
    out = {'host': platform.processor() or platform.machine(), 'threads': 1, 'mode': 'eval',
           'cases': {}}
    for gen, n_img, reps in (('planted', 64, 2), ('uniform', 8, 1)):
        ref_ms, orc_ms = [], []
        for seed in range(n_img):
            cif, caf = synthetic.generate(gen, 80, 80, seed)
            cc = dec.CifCaf(dec.FieldConfig(), keypoints=constants.COCO_KEYPOINTS, skeleton=skel)
            ref_ms.append(med_ms(lambda: cc([cif, caf]), reps))
            orc_ms.append(med_ms(lambda: oracle.decode(cif, caf, skel, cfg), reps))
        r, o = float(np.median(ref_ms)), float(np.median(orc_ms))
        # throughput ratio: total reference time over total oracle time on the same images
        rt, ot = float(np.sum(ref_ms)), float(np.sum(orc_ms))
        out['cases'][gen] = {'images': n_img, 'reference_ms_per_image': round(r, 3),
                             'oracle_ms_per_image': round(o, 3), 'ratio': round(rt / ot, 3),
                             'ratio_of_medians': round(r / o, 3),
                             'reference_ms_total': round(rt, 1), 'oracle_ms_total': round(ot, 1)}
        print(gen, out['cases'][gen], flush=True)
    with open(os.path.join(REPO, 'profiles', 'cpu_ratio.json'), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
