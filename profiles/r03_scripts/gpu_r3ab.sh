#!/bin/bash
# Round-3: world-1 sharded step with the overlapped sweep: hardware queues / stream sharing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
B="python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
for rep in 1 2; do
MASTER_PORT=2959$rep step r3ab_ser_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ab_ser_$rep.log
MASTER_PORT=2958$rep NCF_SHARD_OVERLAP_SWEEP=1 step r3ab_ov_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ab_ov_$rep.log
MASTER_PORT=2957$rep NCF_SHARD_OVERLAP_SWEEP=1 GPU_MAX_HW_QUEUES=8 step r3ab_ovq8_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ab_ovq8_$rep.log
MASTER_PORT=2956$rep NCF_SHARD_OVERLAP_SWEEP=1 NCF_SHARD_SWEEP_ON_PLAN=1 step r3ab_ovplan_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ab_ovplan_$rep.log
done
MASTER_PORT=29550 NCF_SHARD_OVERLAP_SWEEP=1 NCF_SHARD_SWEEP_ON_PLAN=1 step r3ab_tests 300 python3 -u -m pytest tests/test_gpu_parity.py -k "sharded_step_world1" -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ab_tests.log
