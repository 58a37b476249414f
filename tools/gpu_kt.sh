# Quick per-kernel timing of the bench (rocprofv3 kernel trace + stats only).
# Usage (on the GPU box): bash tools/gpu_kt.sh <tag> [bench args...]
set -u
TAG=${1:-kt}
shift || true
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/kt_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/err.log" || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for row in csv.DictReader(open(f)):
    print('{:45s} {:5s} {:10.1f} us avg {:8.1f} us total/step'.format(
        row['Name'][:45], row['Calls'], float(row['AverageNs']) / 1e3,
        float(row['TotalDurationNs']) / 1e3 / 12))
PY
