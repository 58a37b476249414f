# GPU checkpoint: the full GPU suite (printing per-case deviations) and smoke.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-r02c}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider -s -rf \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { grep -E "Error|assert|FAILED|failed" gpurun_out/${T}_tests.log | tail -30; exit 1; }
tail -2 gpurun_out/${T}_tests.log
grep -o "max deviation vs reference: .*" gpurun_out/${T}_tests.log | sort | uniq -c | sort -rn | head -5
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
