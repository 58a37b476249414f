# Iteration call: the -m gpu tests (TESTS=0 skips them), then the default bench line without
# the CPU leg.  Usage (via gpurun): bash tools/gpu_iter.sh <tag>
set -u
TAG=${1:-iter}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json \
  2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
