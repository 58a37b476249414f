# A/B timing of library variants (PP_LIB_VARIANT) on the planted and uniform benches.
# Usage: bash tools/gpu_variants.sh tag variant...   ('' = product library)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=$1; shift
for V in "" "$@"; do
  for G in planted uniform; do
    PP_LIB_VARIANT=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-uniform \
      --no-multi --no-configs --generator $G > gpurun_out/${T}_${V}_$G.json 2> gpurun_out/${T}_${V}_$G.err || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/${T}_${V}_$G.json').read().strip().splitlines()[-1])
print('[$V] $G', d['value'], d['ms_per_step'], d['stage_ms'])"
  done
done
