# C5 scoring: per-stage times (before: abl/base.so; after: the in-tree library) and the scoring tests
set -o pipefail
mkdir -p gpurun_out
NCF_HIP_LIB=$PWD/abl/base.so timeout -k 10 300 python -u tools/score_bench.py > gpurun_out/score_base.log 2>&1 || { tail -20 gpurun_out/score_base.log; exit 1; }
timeout -k 10 300 python -u tools/score_bench.py > gpurun_out/score_new.log 2>&1 || { tail -20 gpurun_out/score_new.log; exit 1; }
echo "--- base"; tail -12 gpurun_out/score_base.log; echo "--- new"; tail -12 gpurun_out/score_new.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "scor or graphed or topk or kth" --timeout 200 --timeout-method thread > gpurun_out/score_tests.log 2>&1
rc=$?; tail -3 gpurun_out/score_tests.log; exit $rc
