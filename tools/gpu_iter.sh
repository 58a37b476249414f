# A/B of library variants on one box: CifHr entry points on the uniform and the planted
# batch, each variant twice in alternation.  Usage (via gpurun): bash tools/gpu_iter.sh <variant> ...  ('' = product)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    [ "$v" = "-" ] && v=""
    for G in uniform planted; do
      PP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/hr_time.py $G 256 > gpurun_out/hr_$v.log 2>&1 || exit $?
      echo "variant=$v $G"; grep pp_cifhr gpurun_out/hr_$v.log
    done
  done
done
