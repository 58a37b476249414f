# Seed-loop iteration: decode parity subset, short benches (planted / uniform), seed-loop
# stamps.  Usage: bash tools/gpu_seed_iter.sh [tag]
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-seed}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factory.py -x -q -m gpu \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 \
  || { grep -E "Error|assert|FAILED|failed" gpurun_out/${T}_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for G in planted uniform; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-uniform --no-multi \
    --no-configs --generator $G > gpurun_out/${T}_b_$G.json 2> gpurun_out/${T}_b_$G.err || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/${T}_b_$G.json').read().strip().splitlines()[-1])
print('$G', d['value'], d['ms_per_step'], d['stage_ms'])"
done
PP_LIB_VARIANT=stamps PP_STAMPS_OUT=gpurun_out/${T}_stamps.bin timeout -k 10 200 python tools/stamps_run.py \
  > gpurun_out/${T}_stamps.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${T}_stamps.txt | head -40
