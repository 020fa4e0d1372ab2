# round-5 evidence: the GPU suite, the world-1 row-sharded line, the kernel-trace profile and the
# HBM counters of the C2 step (profiles/r05o_*)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05o}
bash tools/gpu_run.sh $T tests; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_run.sh $T sharded prof pmc
