# the fused-apply bitwise test, then the C2 step at rolling-sweep periods 64 / 128 / 256
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5za}
bash tools/gpu_run.sh $T "t:fused_apply or early_reduce or deterministic" || exit $?
timeout -k 10 600 python -u tools/step_ab.py --reps 3 s64=sweep:64 s128=sweep:128 \
  s256=sweep:256 > gpurun_out/${T}_step_ab.log 2>&1
