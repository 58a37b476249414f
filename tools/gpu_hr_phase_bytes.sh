# FETCH_SIZE / WRITE_SIZE of the decoder CifHr kernel, whole and phase 1 only
# (libpifpaf_amd_exp_phase1.so: python -m openpifpaf_amd.build --exp_phase1).
# Usage (via gpurun): bash tools/gpu_hr_phase_bytes.sh <planted|uniform> <outdir-name>
set -u
R="$GRAFT_REPO_ROOT"
KIND=${1:-planted}
OUT="$R/gpurun_out/${2:-hr_phase}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for V in "" exp_phase1; do
  for C in FETCH_SIZE WRITE_SIZE; do
    PP_LIB_VARIANT=$V timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/${V:-full}_$C" -o run --output-format csv -- python3 $R/tools/hr_run.py $KIND 256 sparse > "$OUT/${V:-full}_$C.log" 2>&1 || { tail -5 "$OUT/${V:-full}_$C.log"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
for v in ('full', 'exp_phase1'):
    for c in ('FETCH_SIZE', 'WRITE_SIZE'):
        per = collections.defaultdict(float)
        for f in glob.glob(out + '/{}_{}/**/*counter_collection.csv'.format(v, c), recursive=True):
            for row in csv.DictReader(open(f)):
                if 'cifhr_sparse' in row['Kernel_Name']:
                    per[row['Dispatch_Id']] += float(row['Counter_Value'])
        vals = list(per.values())
        print(v, c, 'launches', len(vals), 'KB per launch', sum(vals) / max(1, len(vals)))
PY
