# C5 graphed: the threshold sample's expected candidates per user (512 / 384 / 256), interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zg}
for rep in 1 2; do
  for c in 512 256 384; do
    echo "--- SAMPLE_CANDS=$c ($rep)" >> gpurun_out/${T}_c5.log
    timeout -k 10 200 python -u tools/score_bench.py --graph --reps 3 --set scoring.SAMPLE_CANDS=$c \
      >> gpurun_out/${T}_c5.log 2>&1 || exit $?
  done
done
