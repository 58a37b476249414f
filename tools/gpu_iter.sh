# Quick GPU iteration: CifHr/decode parity subset, then the default bench (no uniform /
# multi / CPU legs) and the CifHr stamps timeline.  Usage: bash tools/gpu_iter.sh
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider \
  -k "sparse or batch256 or multi_batch or uniform or stage_calls or workspace" \
  --timeout 120 --timeout-method thread > gpurun_out/t_iter.log 2>&1 || { tail -30 gpurun_out/t_iter.log; exit 1; }
tail -2 gpurun_out/t_iter.log
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_iter.json 2> gpurun_out/b_iter.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/b_iter.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], d['stage_ms'], 'frac', d['roofline']['frac'])
print('uniform', d['uniform']['value'], d['uniform']['stage_ms'])
print('multi', {k: (v['value'], v['stage_ms']) for k, v in d['multi'].items()})"
PP_LIB_VARIANT=stamps PP_HR_STAMPS_OUT=gpurun_out/hr_stamps.bin timeout -k 10 200 python tools/hr_stamps.py > gpurun_out/hr_stamps.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/hr_stamps.txt
