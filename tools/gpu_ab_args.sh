# A/B of two library builds on one box: the default library against libpifpaf_amd_<B>.so
# (PP_LIB_VARIANT), alternating, REPS times each.  Usage (via gpurun):
#   bash tools/gpu_ab_args.sh <tag> <variant B[,C...]> <bench args...>
# (tools/gpu_ab.sh: the whole default bench line per variant)
set -u
TAG=$1; B=$2; shift 2
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
for r in $(seq ${REPS:-3}); do
  for v in default ${B//,/ }; do
    if [ $v = default ]; then unset PP_LIB_VARIANT; else export PP_LIB_VARIANT=$v; fi
    line=$(timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-multi --no-configs "$@" 2>>gpurun_out/${TAG}_ab.err) || exit $?
    echo "$v $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); u=d.get("uniform",{}); r=d.get("roofline_decoder_cifhr",{}); print(d["value"], d["ms_per_step"], u.get("value"), "hr_us", r.get("us_per_image"), "hr_u_ms", u.get("stage_ms",{}).get("cifhr"), "cfg5", d.get("cfg5",{}).get("planted",{}).get("value"), d.get("cfg5",{}).get("uniform",{}).get("value"))')" | tee -a $OUT
  done
done
unset PP_LIB_VARIANT
