"""Kernel resource usage (VGPRs, spills, LDS, occupancy) from the compiler remarks:
    python tools/resource_usage.py grow.hip seed_loop_kernel nms_kernel"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import build as b
src, kerns = sys.argv[1], sys.argv[2:]
cmd = [b.HIPCC] + b.CFLAGS + b.FILE_FLAGS.get(src, []) + ['--offload-arch=' + b.ARCH, '-c', b.CSRC + '/' + src, '-o', '/tmp/x.o', '-Rpass-analysis=kernel-resource-usage', '--offload-device-only']
r = subprocess.run(cmd, capture_output=True, text=True)
lines = r.stderr.splitlines()
for i, l in enumerate(lines):
    if 'Function Name' in l and any(k in l for k in kerns):
        blk = [x.split('remark: ')[-1].replace(' [-Rpass-analysis=kernel-resource-usage]', '') for x in lines[i:i+12]]
        print(blk[0].strip(), '|', ' '.join(x.strip() for x in blk[3:] if any(t in x for t in ('VGPRs:', 'Spill', 'LDS', 'Occupancy', 'Scratch'))))
