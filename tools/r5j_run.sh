# step-time A/B of this round's changes + full-size parity evidence
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5j}
timeout -k 10 400 python -u tools/step_ab.py --reps 3 base= nofuse=engine.FUSE_ATTN_TOWER:0 \
  noearly=deferred.EARLY_CATCHUP:0 neither=engine.FUSE_ATTN_TOWER:0,deferred.EARLY_CATCHUP:0 \
  > gpurun_out/${T}_step_ab.log 2>&1 || exit $?
bash tools/gpu_run.sh $T fullsize
