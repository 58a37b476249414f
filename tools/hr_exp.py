"""CifHr stage timing on the cfg3 planted batch (20 launches, HIP events)."""
import os, sys, time, json
import numpy as np, torch
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
from openpifpaf_amd import synthetic, constants
from openpifpaf_amd._abi import EVAL_CONFIG, make_config
from openpifpaf_amd.engine import DecodeEngine
cif, caf = synthetic.batch('planted', 256, 80, 80)
c = torch.from_numpy(cif).cuda(); f = torch.from_numpy(caf).cuda()
cfg = make_config(**EVAL_CONFIG)
eng = DecodeEngine()
for _ in range(3): eng.launch(c, f, constants.COCO_PERSON_SKELETON, cfg, stages=1)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): eng.launch(c, f, constants.COCO_PERSON_SKELETON, cfg, stages=1)
e1.record(); torch.cuda.synchronize()
print('cifhr ms', e0.elapsed_time(e1) / 20)
