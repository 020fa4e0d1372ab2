#!/bin/bash
# Round-2 evidence at the overlapped-sweep HEAD, one GPU call: the default bench line (C2 fp32
# headline + roofline in-step/isolated + CPU baseline, drop-in, bf16, C4, C5), rocprofv3
# kernel-trace stats of the bench (C4 and the CPU baseline left out), the row-sharded world-1
# bench and its trace.  Every GPU step under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step bench_r02c 900 python3 -u bench.py
step prof_r02c 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02c -o run --output-format csv -- python3 bench.py --no-c4 --no-cpu-baseline --no-dropin
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
step shard_r02c 400 python3 -u bench.py --sharded --no-cpu-baseline --no-score
step profshard_r02c 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profshard_r02c -o run --output-format csv -- python3 bench.py --sharded --steps 50 --warmup 140 --no-cpu-baseline --no-score
echo done
