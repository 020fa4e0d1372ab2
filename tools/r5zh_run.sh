# C5 graphed top-10: kernel trace of the replays (where the 0.2 ms above the kernel sum goes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zh}
rm -rf gpurun_out/${T}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- \
  python3 tools/score_bench.py --graph --k 10 --reps 3 > gpurun_out/${T}_prof.log 2>&1
