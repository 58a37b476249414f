# rocprofv3 kernel trace of the planted cfg3 bench, overlapped (default) and one step at a
# time (--no-overlap).  Usage (via gpurun): bash tools/gpu_kt_cfg3.sh <tag> [extra env]
set -u
TAG=${1:-kt}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/kt3_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
COMMON="--no-cpu-baseline --no-uniform --no-multi --no-configs --steps 12 --warmup 2"
for M in overlap serial; do
  X=""; [ $M = serial ] && X="--no-overlap"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$M" -o run --output-format csv \
    -- python3 "$R/bench.py" $COMMON $X > "$OUT/${M}_bench.json" 2> "$OUT/${M}.err" || exit $?
  python3 - "$OUT" "$M" <<'PY'
import csv, json, sys
out, m = sys.argv[1], sys.argv[2]
d = json.load(open('%s/%s_bench.json' % (out, m)))
print(m, d['value'], d['ms_per_step'], d['stage_ms'])
for r in csv.DictReader(open('%s/%s/run_kernel_stats.csv' % (out, m))):
    n = r['Name'].split('(')[0].replace('void ', '').replace('pp::', '')
    if n.startswith('at::') or 'rocclr' in n:
        continue
    print('  %-40s %5s %9.1f us' % (n[:40], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
