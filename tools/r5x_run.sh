# early dense reductions on the sweep's side stream: the bitwise tests, then the C2 step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5x}
bash tools/gpu_run.sh $T "t:bitwise or sharded or deterministic" || exit $?
timeout -k 10 600 python -u tools/step_ab.py --reps 3 early=trainer.EARLY_REDUCE:1 \
  noearly=trainer.EARLY_REDUCE:0 > gpurun_out/${T}_step_ab.log 2>&1
