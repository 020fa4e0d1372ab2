# one-stage reductions up to 256 partials (NCF_REDUCE_ONE_STAGE): the deterministic / bitwise /
# parity tests, then the C2 step against the HEAD library (ab_lib/libncf_hip_old.so), alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zp}
bash tools/gpu_run.sh $T "t:deterministic or bitwise or matches or vs_oracle or reduce" || exit $?
for rep in 1 2 3; do
  for lib in ab_lib/libncf_hip_old.so neural-collaborative-filtering-demo_amd/libncf_hip.so; do
    echo "--- $lib ($rep)" >> gpurun_out/${T}_ab.log
    NCF_HIP_LIB=$lib timeout -k 10 300 python -u tools/step_ab.py --reps 1 base=trainer.FUSE_APPLY:1 \
      >> gpurun_out/${T}_ab.log 2>&1 || exit $?
  done
done
