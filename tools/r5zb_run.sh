# late catch-up: the bitwise tests, then the C2 step A/B (late on / off) and the sweep period
# at steady state (64 / 128)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zb}
bash tools/gpu_run.sh $T "t:late_catchup or fused_apply or pipelined or deferred or clock" || exit $?
timeout -k 10 900 python -u tools/step_ab.py --reps 3 late=deferred.LATE_CATCHUP:1 \
  nolate=deferred.LATE_CATCHUP:0 late128=deferred.LATE_CATCHUP:1,sweep:128 \
  > gpurun_out/${T}_step_ab.log 2>&1
