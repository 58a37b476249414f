# B-first (force-complete sets before the CifHr map) with capped grids: library variants x
# forced order, planted and uniform.  Usage: bash tools/gpu_bfirst_ab.sh tag variant...
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=$1; shift
for V in "" "$@"; do
  for B in 1 0; do
    for G in planted uniform; do
      PP_LIB_VARIANT=$V PP_PIPE_BFIRST=$B timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        --no-uniform --no-multi --no-configs --generator $G > gpurun_out/${T}.json 2> gpurun_out/${T}.err || exit $?
      python -c "
import json; d=json.loads(open('gpurun_out/${T}.json').read().strip().splitlines()[-1])
print('[$V bfirst=$B] $G', d['value'], d['ms_per_step'])"
    done
  done
done
