# the fused-apply reduce at 4 waves per SIMD (apply as a template argument, one table at a time):
# the bitwise tests, then the C2 step against the HEAD library (ab_lib/libncf_hip_old.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zt}
bash tools/gpu_run.sh $T "t:fused_apply or late_catchup or deferred or bitwise or bf16" || exit $?
for rep in 1 2 3; do
  for lib in ab_lib/libncf_hip_old.so neural-collaborative-filtering-demo_amd/libncf_hip.so; do
    echo "--- $lib ($rep)" >> gpurun_out/${T}_ab.log
    NCF_HIP_LIB=$lib timeout -k 10 300 python -u tools/step_ab.py --reps 1 base=trainer.FUSE_APPLY:1 \
      >> gpurun_out/${T}_ab.log 2>&1 || exit $?
  done
done
