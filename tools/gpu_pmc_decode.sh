# SQ counter passes over the decode kernels of a short planted bench run.
# bash tools/gpu_pmc_decode.sh <outdir-name> [generator] [workload]
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${1:-pmc_dec}"
G=${2:-planted}
W=${3:-cfg3}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-uniform --no-multi --no-configs --no-predict --generator $G --workload $W > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        name = row['Kernel_Name']
        if 'pp::' not in name:
            continue
        key = (name.split('(')[0].replace('void ', '')[:40], row['Counter_Name'])
        tot[key] += float(row['Counter_Value'])
        cnt[key] += 1
for k in sorted(tot):
    print('{:40s} {:24s} {:16.0f} per launch'.format(k[0], k[1], tot[k] / cnt[k]))
PY
