#!/bin/bash
# Round-3: where the drop-in (claim path) forks its id sort: beside the forward / at the tower
# backward / at the attention backward.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
for at in mlp_bwd attn_bwd; do
NCF_CLAIM_SORT_AT=$at step r3aj_t_$at 300 python3 -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3aj_t_$at.log
done
for rep in 1 2; do
for at in forward mlp_bwd attn_bwd; do
NCF_CLAIM_SORT_AT=$at step r3aj_${at}_$rep 300 python3 -u tools/dropin_host.py --warmup 150 --steps 300
echo "$at $(grep -v amdgpu gpurun_out/r3aj_${at}_$rep.log | head -2 | tr '\n' ' ')"
done
done
