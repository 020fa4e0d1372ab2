#!/bin/bash
# Round-3 evidence, one GPU call: the GPU suite, the default bench line (C2 + roofline + CPU
# baseline, drop-in, bf16, C4, C5), the driver's command, rocprofv3 kernel-trace stats of the
# bench (C2 legs), PMC FETCH/WRITE passes (tools/pmc_run.sh), the row-sharded world-1 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step tests_r03 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/tests_r03.log
step bench_r03 900 python3 -u bench.py
step driver_r03 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
step prof_r03 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03 -o run --output-format csv -- python3 bench.py --no-c4 --no-cpu-baseline --no-score
f=$(find gpurun_out/prof_r03 -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py "$f" k_gather_ln_gmf -v > gpurun_out/r03_c2_train_step_timeline.txt
find gpurun_out/prof_r03 -name '*kernel_stats.csv' -exec cp {} gpurun_out/r03_c2_train_kernel_stats.csv \;
rm -f "$f"
step pmc_r03 900 bash tools/pmc_run.sh r03
cp profiles/r03_pmc_traffic.json gpurun_out/r03_pmc_traffic.json
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
step shard_r03 400 python3 -u bench.py --sharded --no-cpu-baseline --no-score --no-c4
echo done
