# fault triage of test_group_rows_bitwise_equals_every_row (every launch synchronised, so the
# faulting kernel is named), then the GPU suite with the table apply fused into the embedding
# backward, then the step A/B of that fusion
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5z}
NCF_DEBUG_SYNC=1 bash tools/gpu_run.sh ${T}dbg "t:group_rows_bitwise" || exit $?
bash tools/gpu_run.sh $T tests || exit $?
timeout -k 10 600 python -u tools/step_ab.py --reps 3 fuse=trainer.FUSE_APPLY:1 \
  nofuse=trainer.FUSE_APPLY:0 > gpurun_out/${T}_step_ab.log 2>&1
