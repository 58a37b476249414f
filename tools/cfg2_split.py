"""Diagnostic: cfg2 (one 80x80 image: CifHr + seeds, the decoder's stages 1 | 2) device time
for several split-field settings (PP_SPLIT_SLOTS: workgroups per field = slots / 17).  The
product library ignores PP_SPLIT_SLOTS; it is read by the diagnostic build only
(`python -m openpifpaf_amd.build --stamps`, loaded with PP_LIB_VARIANT=stamps).

    python tools/cfg2_split.py [planted|uniform] [slots ...]
"""
import os
import subprocess
import sys

kind = sys.argv[1] if len(sys.argv) > 1 else 'planted'
settings = [int(v) for v in sys.argv[2:]] or [1024, 512, 256, 128, 64]
for slots in settings:
    # sparse_split reads PP_SPLIT_SLOTS once per process: one child per setting
    code = r'''
import os, sys, torch
sys.path.insert(0, %r)
from openpifpaf_amd import constants, synthetic
from openpifpaf_amd._abi import EVAL_CONFIG, make_config
from openpifpaf_amd.engine import DecodeEngine, STAGE_CIFHR, STAGE_SEEDS
cif, caf = synthetic.batch(%r, 1, 80, 80)
c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
eng = DecodeEngine(); cfg = make_config(**EVAL_CONFIG); sk = constants.COCO_PERSON_SKELETON
for _ in range(20): eng.launch(c, f, sk, cfg, stages=STAGE_CIFHR | STAGE_SEEDS)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200): eng.launch(c, f, sk, cfg, stages=STAGE_CIFHR | STAGE_SEEDS)
e1.record(); torch.cuda.synchronize()
print('slots %d: %%.2f us per call' %% (e0.elapsed_time(e1) / 200 * 1e3))
''' % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), kind, slots)
    env = dict(os.environ, PP_SPLIT_SLOTS=str(slots), PP_LIB_VARIANT='stamps')
    subprocess.run([sys.executable, '-c', code], env=env, check=True, timeout=120)
