# rocprofv3 kernel stats of cfg2 (one 80x80 image, CifHr + seeds) under library variants.
# Usage (via gpurun): bash tools/gpu_cfg2_variants.sh <variant> ...  ('-' = the product library)
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  for G in planted uniform; do
    OUT="$R/gpurun_out/c2v_${v}_$G"
    PP_LIB_VARIANT=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
      -- python3 "$R/bench.py" --workload cfg2 --generator $G --steps 50 --warmup 5 \
      --no-cpu-baseline > "$OUT.json" 2> "$OUT.err" || exit $?
    python3 -c "
import csv
rows = [r for r in csv.DictReader(open('$OUT/run_kernel_stats.csv')) if 'pp::' in r['Name']]
print('variant=$v $G', ' '.join('%s:%.1f' % (r['Name'].split('(')[0].split('::')[-1][:22], float(r['AverageNs']) / 1e3) for r in rows))
"
  done
done
