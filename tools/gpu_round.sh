# One GPU call for a round checkpoint: parity tests, smoke, the default bench line, then
# the rocprofv3 kernel trace + PMC passes (tools/gpu_profile.sh).  Every GPU step has its
# own time limit and the chain stops at the first failure.
# Usage (via gpurun): bash tools/gpu_round.sh <tag>;  then here: python tools/prof_summary.py <tag>
set -u
TAG=${1:-r01c}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 540 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
[ "${PROFILE:-1}" = "1" ] && bash tools/gpu_profile.sh "$TAG"
true
