# rocprofv3 kernel traces of cfg2 (one 80x80 image, CifHr + seeds), planted and uniform.
# Usage (on the GPU box, via gpurun): bash tools/gpu_profile_cfg2.sh <tag>
set -u
TAG=${1:-r03}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/profc2_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for G in planted uniform; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$G" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload cfg2 --generator $G --steps 50 --warmup 5 \
    --no-cpu-baseline > "$OUT/${G}_bench.json" 2> "$OUT/${G}.err" || exit $?
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$G/run_kernel_stats.csv')):
    print('$G', r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
"
done
