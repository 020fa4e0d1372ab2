#!/bin/bash
# Round-3 evidence, one GPU call: the GPU suite; PMC FETCH/WRITE passes of the C2 step
# (tools/pmc_run.sh) and of the C5 scan (score_bench) first, so the bench lines carry this
# build's traffic; the default bench line (C2 + roofline + CPU baseline, drop-in, bf16, C4, C5);
# the driver's command; rocprofv3 kernel-trace stats of the C2 legs and one step's per-queue
# timeline; the row-sharded world-1 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step tests_r03 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/tests_r03.log
step pmc_r03 900 bash tools/pmc_run.sh r03
cp profiles/r03_pmc_traffic.json gpurun_out/r03_pmc_traffic.json
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_c5_$C 300 rocprofv3 --pmc $C -d gpurun_out/pmc_c5_$C -o run --output-format csv -- python3 tools/score_bench.py --reps 1
done
python3 tools/pmc_traffic.py gpurun_out/pmc_c5_FETCH_SIZE gpurun_out/pmc_c5_WRITE_SIZE profiles/r03_c5_pmc_traffic.json > gpurun_out/r03_c5_pmc.txt
cp profiles/r03_c5_pmc_traffic.json gpurun_out/r03_c5_pmc_traffic.json
step bench_r03 900 python3 -u bench.py
step driver_r03 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
step prof_r03 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03 -o run --output-format csv -- python3 bench.py --no-c4 --no-cpu-baseline --no-score
f=$(find gpurun_out/prof_r03 -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py "$f" k_gather_ln_gmf -v > gpurun_out/r03_c2_train_step_timeline.txt
find gpurun_out/prof_r03 -name '*kernel_stats.csv' -exec cp {} gpurun_out/r03_c2_train_kernel_stats.csv \;
rm -f "$f"
step tl_r03 300 rocprofv3 --kernel-trace -d gpurun_out/tl_r03 -o run --output-format csv -- python3 tools/kernel_ab.py --warmup 140 --steps 200
f=$(find gpurun_out/tl_r03 -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.5 > gpurun_out/r03_c2_fused_step_queues.txt
rm -f "$f"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
step shard_r03 400 python3 -u bench.py --sharded --no-cpu-baseline --no-score --no-c4
echo done
