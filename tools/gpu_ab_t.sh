# parity tests, the stamps diagnostics (if the stamps library is built), then tools/gpu_ab.sh
# over the given variants.
# Usage (via gpurun): bash tools/gpu_ab_t.sh <tag> <variants...>
set -u
TAG=$1
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
if [ "${STAMPS:-0}" = "1" ]; then
  PP_LIB_VARIANT=stamps PP_STAMPS_OUT=gpurun_out/${TAG}_st.bin timeout -k 10 200 \
    python -u tools/stamps_run.py planted:256:80 > gpurun_out/${TAG}_stamps.txt 2>&1 || exit $?
  rm -f gpurun_out/${TAG}_st.bin
  head -22 gpurun_out/${TAG}_stamps.txt
fi
bash tools/gpu_ab.sh "$@"
