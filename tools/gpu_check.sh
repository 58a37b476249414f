# One GPU call for an iteration: the -m gpu parity tests, then (if green) the cfg2 kernel
# profile and the default bench line without the CPU leg.
# Usage (via gpurun): bash tools/gpu_check.sh <tag> [pytest -k expression]
set -u
TAG=${1:-chk}
K=${2:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$K" ]; then SEL=(-k "$K"); else SEL=(); fi
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu "${SEL[@]}" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile_cfg2.sh "$TAG" || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-multi > gpurun_out/${TAG}_bench.json \
  2> gpurun_out/${TAG}_bench.err || exit $?
python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open('gpurun_out/%s_bench.json' % sys.argv[1]))
print(d['value'], d['ms_per_step'], d['stage_ms'])
for k in ('uniform', 'cfg2', 'cfg5', 'roofline', 'roofline_uniform'):
    print(k, d.get(k))
PY
# KT=1: also a rocprofv3 kernel trace of the default (overlapped) bench (tools/timeline.py)
if [ "${KT:-0}" = "1" ]; then
  R="$GRAFT_REPO_ROOT"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_$TAG" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-uniform --no-multi --no-configs \
    > "$R/gpurun_out/kt_${TAG}_bench.json" 2> "$R/gpurun_out/kt_${TAG}.err" || exit $?
  echo kernel trace done
fi
# KTU=1: the same for the uniform generator (cfg3 uniform, 6 steps)
if [ "${KTU:-0}" = "1" ]; then
  R="$GRAFT_REPO_ROOT"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ktu_$TAG" -o run --output-format csv \
    -- python3 "$R/bench.py" --generator uniform --steps 6 --warmup 2 --no-cpu-baseline --no-uniform --no-multi --no-configs \
    > "$R/gpurun_out/ktu_${TAG}_bench.json" 2> "$R/gpurun_out/ktu_${TAG}.err" || exit $?
  echo uniform kernel trace done
fi
