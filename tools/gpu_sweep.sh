set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/sweep_bench > gpurun_out/sweep1.log 2>&1
cat gpurun_out/sweep1.log
if [ -n "$PMC" ]; then
timeout -k 10 120 rocprofv3 --pmc $PMC -d gpurun_out/sweep_pmc -o run --output-format csv -- ./tools/sweep_bench > gpurun_out/sweep_pmc.log 2>&1
fi
