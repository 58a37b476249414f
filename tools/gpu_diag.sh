# Diagnostics in one GPU call: grow-kernel stamps (stamps build) and a kernel trace of the
# default overlapped bench, plus the default bench line without the CPU leg.
# Usage (via gpurun): bash tools/gpu_diag.sh <tag> [stamps cases...]
set -u
TAG=${1:-diag}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
if [ -f openpifpaf_amd/libpifpaf_amd_stamps.so ]; then
  PP_LIB_VARIANT=stamps PP_STAMPS_OUT=gpurun_out/${TAG}_stamps.bin timeout -k 10 200 \
    python -u tools/stamps_run.py "$@" > gpurun_out/${TAG}_stamps.txt 2>&1 || exit $?
  rm -f gpurun_out/${TAG}_stamps.bin
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-multi > gpurun_out/${TAG}_bench.json \
  2> gpurun_out/${TAG}_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-uniform --no-multi --no-configs \
  > "$R/gpurun_out/kt_${TAG}_bench.json" 2> "$R/gpurun_out/kt_${TAG}.err" || exit $?
echo diag done
