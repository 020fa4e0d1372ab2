# C5 scoring A/B over environment settings: bash tools/gpu_score_env.sh "NAME=V ..." "NAME=V ..." ...
set -o pipefail
mkdir -p gpurun_out
n=0
for e in "$@"; do
  n=$((n+1))
  env $e timeout -k 10 300 python -u tools/score_bench.py > gpurun_out/score_env$n.log 2>&1 || { tail -20 gpurun_out/score_env$n.log; exit 1; }
  echo "--- $e"; tail -2 gpurun_out/score_env$n.log
done
