# SQ / TCC counter passes over one CifHr kernel family alone.
# bash tools/gpu_pmc_hr.sh <planted|uniform> <n> <sparse|dense> <outdir-name>
set -u
R="$GRAFT_REPO_ROOT"
KIND=${1:-planted}; N=${2:-256}; WHICH=${3:-sparse}
OUT="$R/gpurun_out/${4:-pmc_hr}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 $R/tools/hr_run.py $KIND $N $WHICH > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if 'cifhr' not in row['Kernel_Name']:
            continue
        key = (row['Kernel_Name'].split('(')[0].split('<')[0], row['Counter_Name'])
        tot[key] += float(row['Counter_Value'])
        cnt[key] += 1
for k in sorted(tot):
    print('{:28s} {:24s} {:16.0f} per launch'.format(k[0], k[1], tot[k] / cnt[k]))
PY
