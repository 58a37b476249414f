# Seed-loop speculation distance sweep (PP_SPEC_FAR, in joint scales): parity once, then
# the planted and uniform benches per setting.  Results never depend on the knob.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for F in ${PP_SWEEP:-4 8 12 24}; do
  for G in planted uniform; do
    PP_SPEC_FAR=$F timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --generator $G --no-cpu-baseline > gpurun_out/sweep_${F}_$G.json 2> gpurun_out/sweep_${F}_$G.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/sweep_${F}_$G.json'));print('far=$F $G', d['value'], d['stage_ms'])"
  done
done
