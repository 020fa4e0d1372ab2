#!/bin/bash
# HBM traffic per kernel: two separate rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE) over a
# short bench run, then tools/pmc_traffic.py -> profiles/<tag>_pmc_traffic.json.
#   bash tools/pmc_run.sh r01            (PMC_CMD: the profiled program; default a short C2 bench)
set -e
TAG=${1:-r01}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/pmc_$C -o run --output-format csv -- \
    ${PMC_CMD:-python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-score --infer-pairs 64} > gpurun_out/pmc_$C.log 2>&1
done
python3 tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE \
  profiles/${TAG}_pmc_traffic.json
