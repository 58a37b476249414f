# Round-6 first GPU call: every GPU test (with the cfg4 eight-rank test), the cfg4 gloo
# rehearsal bench (8 ranks on one GPU, 2048 images), then the default bench line.
set -u
TAG=${1:-r06a}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --gpus 8 --backend gloo --workload cfg4 --no-uniform \
  --no-multi --no-configs --no-cpu-baseline > gpurun_out/${TAG}_bench_gloo8.json \
  2> gpurun_out/${TAG}_bench_gloo8.err || exit $?
cat gpurun_out/${TAG}_bench_gloo8.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json \
  2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
