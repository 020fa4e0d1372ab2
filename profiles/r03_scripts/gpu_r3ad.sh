#!/bin/bash
# Round-3: one side stream for the id sort and the overlapped sweep (fused step, drop-in).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3ad_tests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ad_tests.log
NCF_SHARE_SIDE=1 step r3ad_tests_share 600 python3 -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "hooked or tapes or deferred or fused or pipelined or dedup" -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ad_tests_share.log
B="python3 -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-score --no-c4"
for rep in 1 2 3; do
step r3ad_def_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ad_def_$rep.log
NCF_SHARE_SIDE=1 step r3ad_share_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ad_share_$rep.log
done
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29544
step r3ad_shard 300 python3 -u bench.py --sharded --steps 300 --warmup 20 --no-cpu-baseline --no-score --no-c4 && python3 tools/bench_summ.py gpurun_out/r3ad_shard.log
