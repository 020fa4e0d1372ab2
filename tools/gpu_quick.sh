#!/bin/bash
# GPU check used between commits: the -m gpu suite, then a short bench (no C4 / CPU baseline).
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; tail -4 gpurun_out/q_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/q_tests.log | head -30; exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 100 --warmup 140 --no-c4 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/q_bench.log > gpurun_out/q_bench.json || tail -20 gpurun_out/q_bench.log
exit $rc
