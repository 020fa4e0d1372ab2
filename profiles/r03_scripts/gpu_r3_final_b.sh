#!/bin/bash
# Round-3 closing evidence, call B: PMC FETCH/WRITE passes of the C2 step and the C5 scan,
# rocprofv3 kernel-trace stats of the C2 legs, one step's per-queue timeline, and the
# row-sharded world-1 bench line, at HEAD.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step test_train_resume 300 python3 -u -m pytest tests/test_gpu_dropin.py -k "train_epochs_checkpoints" -x -q --timeout 200 --timeout-method thread
step pmc_r03 400 bash tools/pmc_run.sh r03
cp profiles/r03_pmc_traffic.json gpurun_out/r03_pmc_traffic.json
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_c5_$C 200 rocprofv3 --pmc $C -d gpurun_out/pmc_c5_$C -o run --output-format csv -- python3 tools/score_bench.py --reps 1
done
python3 tools/pmc_traffic.py gpurun_out/pmc_c5_FETCH_SIZE gpurun_out/pmc_c5_WRITE_SIZE profiles/r03_c5_pmc_traffic.json > gpurun_out/r03_c5_pmc.txt
cp profiles/r03_c5_pmc_traffic.json gpurun_out/r03_c5_pmc_traffic.json
step prof_r03 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03 -o run --output-format csv -- python3 bench.py --no-c4 --no-cpu-baseline --no-score
f=$(find gpurun_out/prof_r03 -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py "$f" k_gather_ln_gmf -v > gpurun_out/r03_c2_train_step_timeline.txt
find gpurun_out/prof_r03 -name '*kernel_stats.csv' -exec cp {} gpurun_out/r03_c2_train_kernel_stats.csv \;
rm -f "$f"
step prof_c5_r03 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_r03 -o run --output-format csv -- python3 tools/score_bench.py --reps 3
find gpurun_out/prof_c5_r03 -name '*kernel_stats.csv' -exec cp {} gpurun_out/r03_c5_kernel_stats.csv \;
find gpurun_out/prof_c5_r03 -name '*kernel_trace.csv' -delete
step tl_r03 200 rocprofv3 --kernel-trace -d gpurun_out/tl_r03 -o run --output-format csv -- python3 tools/kernel_ab.py --warmup 140 --steps 200
f=$(find gpurun_out/tl_r03 -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" k_gather_ln_gmf 0.5 > gpurun_out/r03_c2_fused_step_queues.txt
rm -f "$f"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
step shard_r03 300 python3 -u bench.py --sharded --no-cpu-baseline --no-score --no-c4
echo done
