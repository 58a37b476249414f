# Round-end evidence in one GPU call: the round checkpoint (parity tests, smoke, default
# bench line, kernel trace + PMC passes of cfg3), then the dense-workload and cfg2 traces.
# Usage (via gpurun): bash tools/gpu_final.sh <tag>
set -u
TAG=${1:-r03n}
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh "$TAG" || exit $?
bash tools/gpu_profile_dense.sh "$TAG" || exit $?
bash tools/gpu_profile_cfg2.sh "$TAG" || exit $?
echo final done
