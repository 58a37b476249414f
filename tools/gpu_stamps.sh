# Grow-kernel stamps (the diagnostic build, libpifpaf_amd_stamps.so) of the planted and
# uniform cfg3 batches, one decode at a time.  Usage (via gpurun): bash tools/gpu_stamps.sh <tag>
set -u
TAG=${1:-stamps}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PP_LIB_VARIANT=stamps PP_STAMPS_OUT=gpurun_out/${TAG}_stamps.bin timeout -k 10 300 \
  python -u tools/stamps_run.py planted:256:80 uniform:32:80 > gpurun_out/${TAG}_stamps.txt 2>&1
rc=$?
cat gpurun_out/${TAG}_stamps.txt
exit $rc
