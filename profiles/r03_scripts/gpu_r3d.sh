#!/bin/bash
# Round-3: fused D=128 tower / attention block (C4) parity, the C4-size exchange, then the full
# GPU suite.  Each GPU step under its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3d_new 400 python3 -u -m pytest tests/test_gpu_parity.py -k "mlp_tower_matches_unfused or attn_block_matches_unfused or attn_block_recompute or shard_exchange or train_vs_oracle" -x -v --timeout 200 --timeout-method thread
grep -E "passed|failed" gpurun_out/r3d_new.log | tail -3
step r3d_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -3 gpurun_out/r3d_tests.log
