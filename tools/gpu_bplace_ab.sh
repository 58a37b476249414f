# Force-complete set placement in DecodePipeline (PP_PIPE_BFIRST = 0 / 1 / lazy), planted
# and uniform, each run twice in alternation.  Usage: bash tools/gpu_bplace_ab.sh tag
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=$1
for R in 1 2; do
  for B in 0 1 lazy; do
    for G in planted uniform; do
      PP_PIPE_BFIRST=$B timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        --no-uniform --no-multi --no-configs --generator $G > gpurun_out/${T}.json 2> gpurun_out/${T}.err || exit $?
      python -c "
import json; d=json.loads(open('gpurun_out/${T}.json').read().strip().splitlines()[-1])
print('[bfirst=$B run $R] $G', d['value'], d['ms_per_step'])"
    done
  done
done
