# C5 scan users in threshold order (scoring.SORT_USERS): the C5 tests, then graphed C5 on / off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zk}
bash tools/gpu_run.sh $T "t:sample or score or topk or scan" || exit $?
for rep in 1 2; do
  for v in 0 1; do
    echo "--- SORT_USERS=$v ($rep)" >> gpurun_out/${T}_c5.log
    timeout -k 10 200 python -u tools/score_bench.py --graph --reps 3 --set scoring.SORT_USERS=$v \
      >> gpurun_out/${T}_c5.log 2>&1 || exit $?
  done
done
