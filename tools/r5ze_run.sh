# the side-stream join after the flat Adam (trainer.SPLIT_CLOSE): bitwise tests, then the A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5ze}
bash tools/gpu_run.sh $T "t:late_catchup or fused_apply or pipelined or deferred or clock or graph" || exit $?
timeout -k 10 900 python -u tools/step_ab.py --reps 3 split=trainer.SPLIT_CLOSE:1 \
  nosplit=trainer.SPLIT_CLOSE:0 > gpurun_out/${T}_step_ab.log 2>&1
