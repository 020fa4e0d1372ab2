set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sharded_step_world1 or emulated_ranks" -x -q --timeout 200 --timeout-method thread > gpurun_out/sh_tests.log 2>&1 || { tail -30 gpurun_out/sh_tests.log; exit 1; }
tail -3 gpurun_out/sh_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 250 --timeout-method thread > gpurun_out/sh_tests2.log 2>&1 || { tail -30 gpurun_out/sh_tests2.log; exit 1; }
tail -3 gpurun_out/sh_tests2.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u bench.py --sharded --steps 200 --warmup 140 --no-cpu-baseline --no-score --no-c4 > gpurun_out/sh_bench.log 2>&1
grep '^{' gpurun_out/sh_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('kernel_ms_per_step'))"
