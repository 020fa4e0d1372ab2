# early catch-up + fused attention/tower: the bitwise tests, full-size parity (a plain test
# failure, rc 1, does not stop the run; any other status does), the GPU suite, short bench,
# per-launch times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5h}
bash tools/gpu_run.sh $T "t:early_catchup" || exit $?
bash tools/gpu_run.sh $T fullsize; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_run.sh $T tests; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_run.sh $T quick &&
timeout -k 10 300 python -u tools/tower_ab.py > gpurun_out/${T}_tower_ab.log 2>&1
