#!/bin/bash
# SQ counters of the step's kernels (one rocprofv3 pass per counter group), for stall analysis:
#   bash tools/pmc_sq.sh [tag]   ->  gpurun_out/sq<tag>_<i>/...csv ; summary by tools/pmc_sq_summary.py
#   SQ_CMD: the profiled program (default: the C2 step through tools/kernel_ab.py)
set -e
mkdir -p gpurun_out
TAG=${1:-}
export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C -d gpurun_out/sq${TAG}_$i -o run --output-format csv -- \
    ${SQ_CMD:-python3 tools/kernel_ab.py --warmup 3 --steps 3} > gpurun_out/sq${TAG}_$i.log 2>&1
done
