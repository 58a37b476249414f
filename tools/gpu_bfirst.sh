# A/B of the force-complete set placement in DecodePipeline (engine._B_FIRST): default
# (auto), 0, 1 and lazy (gated, on the tail stream after the seed loop), planted and uniform.
# Usage (via gpurun): bash tools/gpu_bfirst.sh <tag>
set -u
TAG=${1:-bf}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for G in planted uniform; do
  ST=20; [ $G = uniform ] && ST=6
  for M in auto 0 1 lazy; do
    if [ $M = auto ]; then E=""; else E="PP_PIPE_BFIRST=$M"; fi
    env $E timeout -k 10 200 python -u bench.py --generator $G --steps $ST --warmup 2 \
      --no-cpu-baseline > gpurun_out/${TAG}_${G}_${M}.json 2> gpurun_out/${TAG}_${G}_${M}.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_${G}_${M}.json')); print('$G', '$M', d['ms_per_step'], d['stage_ms'])"
  done
done
