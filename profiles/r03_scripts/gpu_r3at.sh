#!/bin/bash
# Round-3: one-product bf16 scan for C5 (margin 4e-3 |q| max|p|, fp32 re-scoring) vs two terms.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3at_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -k "scor or topk or score or split" -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3at_tests.log
NCF_SCORE_TERMS=1 step r3at_tests1 400 python3 -u -m pytest tests/test_gpu_parity.py -k "scor or topk or score or split" -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3at_tests1.log
for rep in 1; do
for t in 2 1; do
NCF_SCORE_TERMS=$t step r3at_t${t}_$rep 200 python3 -u tools/score_bench.py --reps 3
echo "terms=$t: $(grep -v amdgpu gpurun_out/r3at_t${t}_$rep.log | grep '^k=' | cut -c1-200 | tr '\n' ' ')"
done
done
