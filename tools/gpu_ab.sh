# A/B of library variants on one box (openpifpaf_amd.build VARIANTS; '-' = the product):
# the default bench line without the CPU leg, each variant twice in alternation.
# Usage (via gpurun): bash tools/gpu_ab.sh <tag> - base noself PP_PIPE_BFIRST=lazy ...
# (an item with '=' is an environment setting for the product library; several joined by ',')
set -u
TAG=$1
shift
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    lv="$v"; ev="PP_AB_NONE=1"
    [ "$v" = "-" ] && lv=""
    case "$v" in *=*) ev="${v//,/ }"; lv="";; esac
    env $ev PP_LIB_VARIANT=$lv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-multi \
      > gpurun_out/ab_${TAG}_${v}_${rep}.json 2> gpurun_out/ab_${TAG}_${v}_${rep}.err || exit $?
    python3 - gpurun_out/ab_${TAG}_${v}_${rep}.json "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c5, c2 = d.get('cfg5', {}), d.get('cfg2', {})
print('{:8s} planted {:8.0f} ({:.4f} ms) uniform {:7.0f} cfg5 p/u {:6.0f} / {:5.0f} cfg2 p/u {} / {} us  hr {:.3f} ms hr_u {:.3f} ms'.format(
    sys.argv[2], d['value'], d['ms_per_step'], d.get('uniform', {}).get('value', 0),
    c5.get('planted', {}).get('value', 0), c5.get('uniform', {}).get('value', 0),
    c2.get('planted', {}).get('us_per_call_device'), c2.get('uniform', {}).get('us_per_call_device'),
    d['roofline']['ms_per_launch'], d.get('roofline_uniform', {}).get('ms_per_launch', 0)))
PY
  done
done
