# C5 scoring: per-stage times with the fp32 MFMA scan (NCF_SCORE_SPLIT=0) and the split-bf16 scan, then the scoring tests
set -o pipefail
mkdir -p gpurun_out
NCF_SCORE_SPLIT=0 timeout -k 10 300 python -u tools/score_bench.py > gpurun_out/score_fp32.log 2>&1 || { tail -20 gpurun_out/score_fp32.log; exit 1; }
timeout -k 10 300 python -u tools/score_bench.py > gpurun_out/score_split.log 2>&1 || { tail -20 gpurun_out/score_split.log; exit 1; }
echo "--- fp32"; tail -12 gpurun_out/score_fp32.log; echo "--- split"; tail -12 gpurun_out/score_split.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "scor or graphed or topk or kth" --timeout 200 --timeout-method thread > gpurun_out/score_tests.log 2>&1
rc=$?; tail -5 gpurun_out/score_tests.log; exit $rc
