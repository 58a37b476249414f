# PMC passes over cfg2 (one 80x80 image, CifHr + seeds): where the small kernels' wave
# cycles go (issue, wait, instruction fetch).  Usage (via gpurun): bash tools/gpu_pmc_cfg2.sh <tag>
set -u
TAG=${1:-c2}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmcc2_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G=${GEN:-planted}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_BUSY_CYCLES"
P2="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$R/bench.py" --workload cfg2 --generator $G --steps 10 --warmup 2 \
    --no-cpu-baseline > "$OUT/p${i}_bench.json" 2> "$OUT/p$i.err" || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')[-40:]
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    print(k, ' '.join('{}={:.0f}'.format(c, sum(v) / len(v)) for c, v in sorted(d.items())))
PY
