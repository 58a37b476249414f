set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider -k "cifhr or sparse or batch or uniform or multi" --timeout 120 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { grep -E "Error|assert|FAILED|failed" gpurun_out/${T}_t.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t.log
PP_LIB_VARIANT=stamps PP_HR_STAMPS_OUT=gpurun_out/hr_stamps.bin timeout -k 10 200 python tools/hr_stamps.py > gpurun_out/${T}_hr.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/${T}_hr.txt | grep -E "==|span|lifetime|phase"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-uniform --no-multi --no-configs > gpurun_out/${T}_b.json 2> gpurun_out/${T}_b.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/${T}_b.json').read().strip().splitlines()[-1]); print('planted', d['value'], d['ms_per_step'], d['stage_ms'])"
