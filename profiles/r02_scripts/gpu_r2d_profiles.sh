#!/bin/bash
# Round-2 session-4 evidence (C5 scoring rework): the GPU suite, the default bench line,
# rocprofv3 kernel-trace stats and PMC HBM traffic of the C5 micro-benchmark.  Every GPU step
# under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step gputests_r02d 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -2 gpurun_out/gputests_r02d.log
step bench_r02d 900 python3 -u bench.py
step profc5_r02d 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5_r02d -o run --output-format csv -- python3 tools/score_bench.py
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_$C 300 rocprofv3 --pmc $C -d gpurun_out/pmc_$C -o run --output-format csv -- python3 tools/score_bench.py --reps 1
done
echo done
