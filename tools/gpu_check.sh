# GPU round trip: parity tests, then (if they ran) the bench and the stamps diagnostic.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit $?
cat gpurun_out/bench1.json
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --generator uniform --no-cpu-baseline > gpurun_out/bench_uniform.json 2> gpurun_out/bench_uniform.err || exit $?
cat gpurun_out/bench_uniform.json
if [ "${PP_STAMPS_RUN:-0}" = "1" ]; then
  rm -f gpurun_out/stamps.bin
  PP_LIB_VARIANT=stamps PP_STAMPS_OUT=gpurun_out/stamps.bin timeout -k 10 300 python tools/stamps_run.py > gpurun_out/stamps.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/stamps.txt
fi
