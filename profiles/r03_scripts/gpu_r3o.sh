#!/bin/bash
# Round-3: launch tapes for the row-sharded step: world-1 bitwise tests, world-2 HIP test, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3o_shard_tests 600 python3 -u -m pytest tests/test_gpu_parity.py -k "sharded or comm or shard_exchange" tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread
tail -12 gpurun_out/r3o_shard_tests.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
step r3o_sharded 400 python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4
grep '^{' gpurun_out/r3o_sharded.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded', d['ms_per_step'])"
export MASTER_PORT=29556 NCF_SHARD_OVERLAP_SWEEP=1
step r3o_sharded_ov 400 python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4
grep '^{' gpurun_out/r3o_sharded_ov.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded overlap', d['ms_per_step'])"
unset NCF_SHARD_OVERLAP_SWEEP
export MASTER_PORT=29557 NCF_TAPE=0
step r3o_sharded_notape 400 python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4
grep '^{' gpurun_out/r3o_sharded_notape.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded notape', d['ms_per_step'])"
