# the owner claim a step ahead: bisect (bitwise vs the fused step), the sharded/dist tests, the
# world-1 sharded line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5v}
timeout -k 10 300 python -u tools/shard_bisect.py > gpurun_out/${T}_bisect.log 2>&1 || exit $?
bash tools/gpu_run.sh $T "t:sharded or dist or comm" sharded
