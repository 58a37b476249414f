# A/B of library variants on one box: the cfg3 bench (planted + uniform legs, no CPU leg)
# and cfg2, each variant twice in alternation.
# Usage (via gpurun): bash tools/gpu_ab_bench.sh <variant> ...  ('-' = the product library)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    [ "$v" = "-" ] && v=""
    PP_LIB_VARIANT=$v timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-multi --no-configs > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
    PP_LIB_VARIANT=$v timeout -k 10 120 python -u bench.py --workload cfg2 --generator uniform \
      --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab2u_$v.json 2> gpurun_out/ab2u_$v.err || exit $?
    PP_LIB_VARIANT=$v timeout -k 10 120 python -u bench.py --workload cfg2 --generator planted \
      --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab2p_$v.json 2> gpurun_out/ab2p_$v.err || exit $?
    python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open('gpurun_out/ab_%s.json' % v))
u = d.get('uniform', {})
c2u = json.load(open('gpurun_out/ab2u_%s.json' % v)); c2p = json.load(open('gpurun_out/ab2p_%s.json' % v))
print('variant=%-6s planted %.4f ms (hr %.4f)  uniform %.3f ms (hr %.3f)  cfg2 u %.4f (hr %.4f) p %.4f (hr %.4f)' % (
    v, d['ms_per_step'], d['stage_ms']['cifhr'], u.get('ms_per_step', 0), u.get('stage_ms', {}).get('cifhr', 0),
    c2u['ms_per_step'], c2u['stage_ms']['cifhr'], c2p['ms_per_step'], c2p['stage_ms']['cifhr']))
PY
  done
done
