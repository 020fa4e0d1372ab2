#!/bin/bash
# Round-3: one-term C5 scan grid: split sizing on/off x minimum rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
for sz in 1 0; do
for r in 2 4 8 16; do
NCF_SCORE_SIZED=$sz NCF_SCORE3_ROUNDS=$r step r3au_${sz}_$r 200 python3 -u tools/score_bench.py --reps 3
echo "sized=$sz rounds=$r: $(grep -v amdgpu gpurun_out/r3au_${sz}_$r.log | grep '^k=' | sed -E 's/ncf_score_(queries|margin|kth)=[0-9.]+ms //g; s/ncf_gemm_f32=[0-9.]+ms //' | cut -c1-120 | tr '\n' ' ')"
done
done
