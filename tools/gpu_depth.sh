set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05d_tests.log; [ $rc -eq 0 ] || exit $rc
for d in 3 4 6 3 4 6; do
  timeout -k 10 120 python -u tools/host_pipe.py --depth $d --steps 100 >> gpurun_out/depth.log 2>&1 || exit $?
done
grep "ms per step\|submit\|blocked" gpurun_out/depth.log
