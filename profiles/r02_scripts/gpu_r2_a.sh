set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_a_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r2_a_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r2_a_bench.log 2>&1
rc=$?
tail -c 3000 gpurun_out/r2_a_bench.log
exit $rc
