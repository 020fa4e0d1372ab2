#!/bin/bash
# Round-2 evidence in one GPU call: rocprofv3 kernel-trace stats of the steady-state bench
# (C2 fp32 + bf16 + C5 lines; C4 and the CPU baseline are separate runs), PMC HBM traffic
# (FETCH_SIZE and WRITE_SIZE in separate passes), the row-sharded world-1 bench and its trace.
# Every GPU step under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step prof_r02 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o run --output-format csv -- python3 bench.py --no-c4 --no-cpu-baseline --no-dropin
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_$C 300 rocprofv3 --pmc $C -d gpurun_out/pmc_$C -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-score --no-c4 --no-dropin --infer-pairs 64
done
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
step shard_r02 400 python3 bench.py --sharded --no-cpu-baseline --no-score
step profshard_r02 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profshard_r02 -o run --output-format csv -- python3 bench.py --sharded --steps 50 --warmup 140 --no-cpu-baseline --no-score
echo done
