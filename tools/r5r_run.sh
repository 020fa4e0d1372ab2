# sharded step (owner gradient sum inside the apply): its tests, the world-1 line; the stream probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5r}
bash tools/gpu_run.sh $T "t:sharded or dist or comm" sharded || exit $?
timeout -k 10 400 python -u tools/stream_probe.py > gpurun_out/${T}_probe.log 2>&1
