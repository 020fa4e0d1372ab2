# round-5 evidence at HEAD: full-size parity, the GPU suite, the driver's bench command, the
# world-1 sharded line, the kernel-trace profile and the HBM counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05y}
bash tools/gpu_run.sh $T fullsize; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # (99: a GPU fault)
bash tools/gpu_run.sh $T tests; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # (99: a GPU fault)
bash tools/gpu_run.sh $T bench sharded prof pmc
