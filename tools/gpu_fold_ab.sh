# CifHr fold variants: bit-exactness of each (the CifHr and stage tests), then the A/B bench.
# Usage (via gpurun): bash tools/gpu_fold_ab.sh <tag> <variant>...   ('-' = the product)
set -u
TAG=$1
shift
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  lv="$v"; [ "$v" = "-" ] && lv=""
  PP_LIB_VARIANT=$lv timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py -k "cifhr or stages_bit_exact or batch_uniform_eval or dense_vs_oracle" \
    > gpurun_out/fold_${TAG}_${v}_tests.log 2>&1 || { tail -30 gpurun_out/fold_${TAG}_${v}_tests.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/fold_${TAG}_${v}_tests.log)"
done
bash tools/gpu_ab.sh "$TAG" "$@"
