# rocprofv3 kernel trace of one bench workload (tools/timeline.py reads it).
# Usage (via gpurun): bash tools/gpu_kt.sh <tag> <bench args...>
set -u
TAG=$1
shift
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu-baseline --no-uniform --no-multi --no-configs "$@" \
  > "$R/gpurun_out/kt_${TAG}_bench.json" 2> "$R/gpurun_out/kt_${TAG}.err" || exit $?
echo "kernel trace $TAG done"
