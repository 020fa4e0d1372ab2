# the row-sharded step's sweep period (64 / 128), then FusedTrainStep's (128 / 256) at steady state
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zo}
bash tools/r5zn_run.sh $T || exit $?
timeout -k 10 900 python -u tools/step_ab.py --reps 3 s128=sweep:128 s256=sweep:256 \
  > gpurun_out/${T}_step_ab.log 2>&1
