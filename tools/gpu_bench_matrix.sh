# the bench across generators / workloads (informational)
set -u
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out
for args in "--generator uniform" "--mode predict" "--workload cfg5" "--workload cfg5 --generator uniform" "--workload cfg2 --steps 50"; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $args >> gpurun_out/bench_matrix.jsonl 2>> gpurun_out/bench_matrix.err || exit $?
done
echo matrix done
