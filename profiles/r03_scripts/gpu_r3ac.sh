#!/bin/bash
# Round-3: world-1 sharded step, serial sweep vs overlapped sweep on the plan stream (3 reps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
B="python3 -u bench.py --sharded --steps 300 --warmup 20 --no-cpu-baseline --no-score --no-c4"
for rep in 1 2 3; do
MASTER_PORT=2959$rep step r3ac_ser_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ac_ser_$rep.log
MASTER_PORT=2956$rep NCF_SHARD_OVERLAP_SWEEP=1 NCF_SHARD_SWEEP_ON_PLAN=1 step r3ac_ovplan_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ac_ovplan_$rep.log
done
unset RANK LOCAL_RANK WORLD_SIZE
NCF_SHARD_OVERLAP_SWEEP=1 NCF_SHARD_SWEEP_ON_PLAN=1 step r3ac_dist 300 python3 -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ac_dist.log
