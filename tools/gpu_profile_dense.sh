# rocprofv3 kernel traces of the dense workloads the default profile (gpu_profile.sh) does
# not cover: cfg3 on the uniform generator, cfg5 (160x160, 44 CAFs, 64 images) planted and
# uniform; each overlapped (the bench default) and one step at a time (--no-overlap), so a
# kernel's own time is separated from the time it spends sharing CUs with the other step.
# Usage (on the GPU box, via gpurun): bash tools/gpu_profile_dense.sh <tag>
# Then here: python tools/prof_dense_summary.py <tag>
set -u
TAG=${1:-r03a}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/profd_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
COMMON="--no-cpu-baseline --no-uniform --no-multi --no-configs"
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv \
    -- python3 "$R/bench.py" $COMMON "$@" > "$OUT/${name}_bench.json" 2> "$OUT/${name}.err" || exit $?
  echo "$name: $(cat "$OUT/${name}_bench.json" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["stage_ms"])')"
}
run cfg3u --generator uniform --steps 6 --warmup 1
run cfg3u_serial --generator uniform --steps 6 --warmup 1 --no-overlap
run cfg5p --workload cfg5 --steps 10 --warmup 1
run cfg5p_serial --workload cfg5 --steps 10 --warmup 1 --no-overlap
run cfg5u --workload cfg5 --generator uniform --steps 4 --warmup 1
run cfg5u_serial --workload cfg5 --generator uniform --steps 4 --warmup 1 --no-overlap
echo profile done
