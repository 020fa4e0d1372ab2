#!/bin/bash
# Round-3: where the world-1 row-sharded step stands (wall, host, GPU kernel sum per step).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
step r3n_sharded 400 python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4
grep '^{' gpurun_out/r3n_sharded.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded', d['ms_per_step'])"
unset RANK LOCAL_RANK WORLD_SIZE
step r3n_shard_host 300 python3 -u tools/shard_host.py --steps 30
grep -v amdgpu.ids gpurun_out/r3n_shard_host.log | head -45
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_PORT=29556
step r3n_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_prof -o run -- python3 -u bench.py --sharded --steps 30 --warmup 5 --no-cpu-baseline --no-score --no-c4 --no-dropin
f=$(find gpurun_out/r3n_prof -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py "$f" k_shard_plan -v | tail -45
