# rocprofv3 kernel trace + stats and separate HBM counter passes for the default bench.
# Usage (on the GPU box, via gpurun): bash tools/gpu_profile.sh <tag>
set -u
TAG=${1:-r01}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o run --output-format csv -- python3 $BENCH > "$OUT/kt_bench.json" 2> "$OUT/kt.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/fetch_bench.json" 2> "$OUT/fetch.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/write_bench.json" 2> "$OUT/write.err" || exit $?
echo profile done
