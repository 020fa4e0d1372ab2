#!/bin/bash
# Round-3: world-1 sharded step, next-batch exchange ahead off (identity at world 1) x sweep overlap.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
B="python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
show() { grep '^{' gpurun_out/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'])"; }
MASTER_PORT=29561 NCF_SHARD_AHEAD=0 step r3q_a0 400 $B && show r3q_a0
MASTER_PORT=29562 NCF_SHARD_AHEAD=0 NCF_SHARD_OVERLAP_SWEEP=1 step r3q_a0_ov 400 $B && show r3q_a0_ov
MASTER_PORT=29563 NCF_SHARD_AHEAD=0 NCF_SHARD_OVERLAP_SWEEP=1 NCF_TAPE=0 step r3q_a0_ov_nt 400 $B && show r3q_a0_ov_nt
MASTER_PORT=29564 step r3q_def 400 $B && show r3q_def
step r3q_fused 400 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4 --no-dropin && show r3q_fused
