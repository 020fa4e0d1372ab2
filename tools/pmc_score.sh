#!/bin/bash
# MFMA-busy and clock counters of the C5 scan kernel (k_collect), one counter pass.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  -d gpurun_out/pmc_score -o run --output-format csv -- python3 tools/score_bench.py --k 10 --reps 1 > gpurun_out/pmc_score.log 2>&1
