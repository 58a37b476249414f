# SQ counter passes over the CifHr sparse kernel alone.  bash tools/gpu_pmc_hr.sh
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc_hr"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 $R/tools/hr_run.py ${1:-planted} ${2:-256} > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(out + '/p*/**/run_counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if 'cifhr_sparse' not in row['Kernel_Name']:
            continue
        tot[row['Counter_Name']] += float(row['Counter_Value'])
        cnt[row['Counter_Name']] += 1
for k in sorted(tot):
    print('{:24s} {:16.0f} per launch'.format(k, tot[k] / cnt[k]))
PY
