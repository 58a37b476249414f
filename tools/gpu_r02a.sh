# First round-2 GPU call: parity tests, smoke, default bench, CifHr timings on both
# generators, kernel trace of the bench, and counter passes of uniform-load CifHr.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-r02a}
timeout -k 10 540 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
cat gpurun_out/${T}_bench.json
for G in planted uniform; do
  timeout -k 10 120 python -u tools/hr_time.py $G 256 > gpurun_out/${T}_hrtime_$G.log 2>&1 || exit $?
  cat gpurun_out/${T}_hrtime_$G.log
done
bash tools/gpu_pmc_hr.sh uniform 256 dense ${T}_pmc_dense_u > gpurun_out/${T}_pmc_dense_u.txt 2>&1 || exit $?
bash tools/gpu_pmc_hr.sh uniform 256 sparse ${T}_pmc_sparse_u > gpurun_out/${T}_pmc_sparse_u.txt 2>&1 || exit $?
cat gpurun_out/${T}_pmc_*_u.txt
