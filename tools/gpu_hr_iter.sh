# CifHr iteration: sparse / dense parity tests, then timings on both generators.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-hr}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
  -k "cifhr or stages_bit_exact or multi_stages or poisoned or batch256 or uniform or cifcaf_vs_oracle or multi_batch or cifdet or add_gauss or multi_unequal" \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { grep -E "Error|assert|FAILED|failed" gpurun_out/${T}_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for G in planted uniform; do
  timeout -k 10 120 python -u tools/hr_time.py $G 256 2>&1 | grep -v amdgpu.ids || exit 1
done
