# the operand-swapped threshold sample (k_sample16t): the C5 tests, then the C5 A/B against the
# HEAD library (ab_lib/libncf_hip_old.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zf}
bash tools/gpu_run.sh $T "t:sample or score or topk or scan" || exit $?
bash tools/gpu_run.sh $T "c5ab:NCF_HIP_LIB=ab_lib/libncf_hip_old.so,neural-collaborative-filtering-demo_amd/libncf_hip.so"
