# A/B of one environment variable on one box: the cfg3 bench (planted + uniform legs, no CPU
# leg), each value twice in alternation ('auto' = unset).
# Usage (via gpurun): bash tools/gpu_env_ab.sh VAR val1 val2 ...
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = "auto" ]; then E=(env -u "$VAR"); else E=(env "$VAR=$v"); fi
    "${E[@]}" timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-multi --no-configs > gpurun_out/env_$v.json 2> gpurun_out/env_$v.err || exit $?
    python3 - "$VAR" "$v" <<'PY'
import json, sys
d = json.load(open('gpurun_out/env_%s.json' % sys.argv[2]))
u = d.get('uniform', {})
print('%s=%-5s planted %.4f ms %s  uniform %.3f ms %s' % (sys.argv[1], sys.argv[2], d['ms_per_step'],
      d['stage_ms'], u.get('ms_per_step', 0), u.get('stage_ms')))
PY
  done
done
