"""Time the seeds stage (emit + sort) of a resident planted / uniform batch with HIP events:
python tools/sort_time.py [planted|uniform] [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, make_config  # noqa: E402
from openpifpaf_amd.engine import STAGE_CIFHR, STAGE_SEEDS, DecodeEngine  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'planted'
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
cif, caf = synthetic.batch(kind, n, 80, 80)
c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
eng = DecodeEngine()
cfg = make_config(**EVAL_CONFIG)
sk = constants.COCO_PERSON_SKELETON
eng.launch(c, f, sk, cfg, stages=STAGE_CIFHR)
for _ in range(3):
    eng.launch(c, f, sk, cfg, stages=STAGE_SEEDS)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    eng.launch(c, f, sk, cfg, stages=STAGE_SEEDS)
e1.record()
torch.cuda.synchronize()
print('{} seeds stage {:.3f} ms'.format(kind, e0.elapsed_time(e1) / 10))
