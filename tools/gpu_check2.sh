# Full GPU parity suite, then the kernel trace of the default bench (tools/gpu_kt.sh).
# Usage (on the GPU box): bash tools/gpu_check2.sh <kt tag>
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu_kt.sh "${1:-x}" || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/kt_${1:-x}/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], d['stage_ms'])
print('roofline', d['roofline'])
print('decoder cifhr', d['roofline_decoder_cifhr'])
print('uniform', d['uniform']['value'], d['uniform']['stage_ms'])
print('multi', {k: (v['value'], v['stage_ms']) for k, v in d['multi'].items()})"
