# A/B of environment settings on the default planted / uniform bench lines.
# Usage: bash tools/gpu_env_ab.sh tag 'ENV=a' 'ENV=b' ...   ('' = unchanged)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=$1; shift
for E in "" "$@"; do
  for G in planted uniform; do
    env $E timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-uniform \
      --no-multi --no-configs --generator $G > gpurun_out/${T}_$G.json 2> gpurun_out/${T}_$G.err || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/${T}_$G.json').read().strip().splitlines()[-1])
print('[$E] $G', d['value'], d['ms_per_step'], d['stage_ms'])"
  done
done
