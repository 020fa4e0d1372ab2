# the sharded step's new launches, forward_simple in training mode, the narrow-D scorer; then the
# world-1 sharded line and the stream-queue probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5s}
bash tools/gpu_run.sh $T "t:sharded or dist or comm or forward_simple_train or narrow_dims" sharded || exit $?
timeout -k 10 400 python -u tools/stream_probe.py > gpurun_out/${T}_probe.log 2>&1
