# dense vs sparse CifHr entry points, planted and uniform (tools/hr_time.py), after the parity subset
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider -k "cifhr or multi" --timeout 120 --timeout-method thread > gpurun_out/hrcmp_t.log 2>&1 || { tail -20 gpurun_out/hrcmp_t.log; exit 1; }
tail -1 gpurun_out/hrcmp_t.log
for G in planted uniform; do
  echo "$G"; timeout -k 10 120 python -u tools/hr_time.py $G 256 || exit $?
done
