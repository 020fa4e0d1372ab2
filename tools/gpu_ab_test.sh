# A/B libraries (tools/ab_libs.sh), then the -m gpu suite against the LAST library given.
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_libs.sh "$@" > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
cat gpurun_out/ab.log
last="${@: -1}"
NCF_HIP_LIB=$PWD/$last timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab_tests.log | head -20; fi
exit $rc
