# round-5 checkpoint: full-size parity, the GPU suite, the driver's bench command (all legs)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5n}
bash tools/gpu_run.sh $T fullsize; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_run.sh $T tests; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_run.sh $T bench
