# C2 step A/B: dense reductions beside the apply, stream priorities
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5p}
timeout -k 10 700 python -u tools/step_ab.py --reps 3 base= redasync=trainer.REDUCE_ASYNC:1 \
  sidehi=deferred.SIDE_PRIORITY:-1 mainhi=prio:-1 red_mainhi=trainer.REDUCE_ASYNC:1,prio:-1 \
  > gpurun_out/${T}_step_ab.log 2>&1
