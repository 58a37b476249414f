# dense CifHr (pp_cifhr) parity and time vs tiles per tile-kernel workgroup (PP_HR_CHUNK)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for C in 32 8 1; do
  PP_HR_CHUNK=$C timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider -k "cifhr" --timeout 120 --timeout-method thread > gpurun_out/chunk_t$C.log 2>&1 || { tail -20 gpurun_out/chunk_t$C.log; exit 1; }
  tail -1 gpurun_out/chunk_t$C.log
done
for C in 32 16 8 4 2 1; do
  echo "chunk $C"; PP_HR_CHUNK=$C timeout -k 10 120 python -u tools/hr_time.py planted 256 || exit $?
done
