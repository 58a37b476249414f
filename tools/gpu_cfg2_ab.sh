# cfg2 (one 80x80 image, CifHr + seeds) device time per call under alternating settings of
# one environment variable.  Usage (via gpurun): bash tools/gpu_cfg2_ab.sh VAR val1 val2 ...
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    for G in planted uniform; do
      env "$VAR=$v" timeout -k 10 120 python -u bench.py --workload cfg2 --generator $G --steps 50 \
        --warmup 5 --no-cpu-baseline > gpurun_out/c2_${v}_$G.json 2> gpurun_out/c2_${v}_$G.err || exit $?
      python3 -c "
import json; d = json.load(open('gpurun_out/c2_${v}_$G.json'))
print('$VAR=$v $G', d.get('us_per_call_device', d.get('ms_per_step')), d.get('us_per_call_host'))"
    done
  done
done
