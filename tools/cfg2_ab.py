"""A/B of library variants on cfg2 (one 80x80 image, CifHr + seeds; bench.cfg2_latency):
each variant in its own process (PP_LIB_VARIANT), alternating, REPS times.

    python tools/cfg2_ab.py <reps> - <variant> [...]      ('-' = the product library)
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import json, sys
sys.path.insert(0, %r)
import bench
from openpifpaf_amd._abi import EVAL_CONFIG, make_config
cfg = make_config(**EVAL_CONFIG)
print(json.dumps({g: bench.cfg2_latency(g, cfg, 'cuda:0') for g in ('planted', 'uniform')}))
''' % REPO

reps, variants = int(sys.argv[1]), sys.argv[2:]
for _ in range(reps):
    for v in variants:
        env = dict(os.environ)
        env.pop('PP_LIB_VARIANT', None)
        if v != '-':
            env['PP_LIB_VARIANT'] = v
        out = subprocess.run([sys.executable, '-c', CODE], env=env, capture_output=True, text=True,
                             timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(out.returncode)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print('{:8s} planted {:7.2f} us  uniform {:7.2f} us'.format(
            v, d['planted']['us_per_call_device'], d['uniform']['us_per_call_device']), flush=True)
