# Round-2 check: new GPU tests (compact records, multi-rank gather), the full GPU suite,
# the default bench, and a 2-rank gloo rehearsal of bench.py --gpus 2 on the one GPU.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-r02b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -k "compact or multirank or sharded" -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_new.log 2>&1 || { tail -40 gpurun_out/${T}_new.log; exit 1; }
tail -3 gpurun_out/${T}_new.log
timeout -k 10 540 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider -s \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 240 python -u bench.py --gpus 2 --backend gloo --steps 10 > gpurun_out/${T}_bench_g2.json 2> gpurun_out/${T}_bench_g2.err || { tail -20 gpurun_out/${T}_bench_g2.err; exit 1; }
cat gpurun_out/${T}_bench_g2.json
