# C5 top-100: the rank-j sample size factor (scoring.RANK_SAMPLE_F 1 / 2 / 3), graphed, interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zl}
bash tools/gpu_run.sh $T "t:topk or rank" || exit $?
for rep in 1 2; do
  for f in 1 2 3; do
    echo "--- RANK_SAMPLE_F=$f ($rep)" >> gpurun_out/${T}_c5.log
    timeout -k 10 200 python -u tools/score_bench.py --graph --reps 3 --k 100 \
      --set scoring.RANK_SAMPLE_F=$f >> gpurun_out/${T}_c5.log 2>&1 || exit $?
  done
done
