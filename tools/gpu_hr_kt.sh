# Kernel trace of the two CifHr entry points (dense pp_cifhr, sparse pp_cifhr_sparse) on a
# resident 256-image batch.  Usage (on the GPU box): bash tools/gpu_hr_kt.sh [planted|uniform]
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/hrkt_${1:-planted}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 "$R/tools/hr_time.py" "${1:-planted}" > "$OUT/hr_time.txt" 2> "$OUT/err.log" || exit $?
cat "$OUT/hr_time.txt"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for row in csv.DictReader(open(f)):
    print('{:50s} {:5s} {:10.1f} us avg'.format(row['Name'][:50], row['Calls'],
                                              float(row['AverageNs']) / 1e3))
PY
