#!/bin/bash
# SQ counters of the step's kernels (one pass per counter group), for stall analysis.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/sq$i -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-score --infer-pairs 64 > gpurun_out/sq$i.log 2>&1
done
