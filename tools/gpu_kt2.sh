# Kernel trace + stats of the bench's decode, planted and uniform (separate runs).
set -u
R="$GRAFT_REPO_ROOT"
T=${1:-r02d}
OUT="$R/gpurun_out/kt_$T"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--steps 10 --warmup 2 --no-cpu-baseline --no-uniform --no-multi --no-configs"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/planted" -o run --output-format csv -- python3 $R/bench.py $B > "$OUT/planted.json" 2> "$OUT/planted.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/uniform" -o run --output-format csv -- python3 $R/bench.py $B --generator uniform > "$OUT/uniform.json" 2> "$OUT/uniform.err" || exit $?
for g in planted uniform; do
  echo "== $g"; f=$(find "$OUT/$g" -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print('%-60s %6s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
done
