# C5 scoring A/B: per-stage times of the in-tree library and of each abl/<name>.so given as arguments
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/score_bench.py > gpurun_out/score_cur.log 2>&1 || { tail -20 gpurun_out/score_cur.log; exit 1; }
echo "--- current"; tail -2 gpurun_out/score_cur.log
for n in "$@"; do
  NCF_HIP_LIB=$PWD/abl/$n.so timeout -k 10 300 python -u tools/score_bench.py > gpurun_out/score_$n.log 2>&1 || { tail -20 gpurun_out/score_$n.log; exit 1; }
  echo "--- $n"; tail -2 gpurun_out/score_$n.log
done
