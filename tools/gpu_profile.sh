# rocprofv3 kernel trace + stats of the default bench, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) of the bench and of the counter-calibration kernels.
# Usage (on the GPU box, via gpurun): bash tools/gpu_profile.sh <tag>
# Summarise afterwards (here): python tools/prof_summary.py <tag>
set -u
TAG=${1:-r01}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 "$R/tools/calib_counters.hip" -o /tmp/calib_counters 2> "$OUT/calib_build.err" || exit $?
python3 -c "import sys; sys.path.insert(0, '$R'); from openpifpaf_amd.build import source_digest; print(source_digest())" > "$OUT/src_sha.txt" || exit $?
BENCH="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-uniform --no-multi --no-configs --no-predict"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- python3 $BENCH > "$OUT/kt_bench.json" 2> "$OUT/kt.err" || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/pmc_$C" -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-uniform --no-multi --no-configs --no-predict > "$OUT/pmc_${C}_bench.json" 2> "$OUT/pmc_$C.err" || exit $?
  timeout -k 10 120 rocprofv3 --pmc $C -d "$OUT/calib_$C" -o run --output-format csv -- /tmp/calib_counters > "$OUT/calib_$C.log" 2>&1 || exit $?
done
echo profile done
