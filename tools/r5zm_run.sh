# C2: the next batch's catch-up queued behind the sort (early, rows of this step locked) against
# behind this step's fused apply (late, the default): the cross-queue wait of the late form
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zm}
bash tools/gpu_run.sh $T "t:early_catchup or late_catchup" || exit $?
timeout -k 10 900 python -u tools/step_ab.py --reps 3 late=deferred.LATE_CATCHUP:1 \
  early=deferred.EARLY_CATCHUP:1,deferred.LATE_CATCHUP:0 > gpurun_out/${T}_step_ab.log 2>&1
