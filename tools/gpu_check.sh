#!/bin/bash
# Run GPU steps in order; each under its own time limit.  Stop at the first step whose exit
# status is not 0/1 (fault, abort, segfault, timeout): nothing more touches the GPU after that.
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  if grep -q "HSA_STATUS_ERROR\|illegal memory access\|MEMORY_APERTURE" "gpurun_out/$name.log"; then
    echo "STOP: $name: the GPU runtime reported a fault"; exit 3
  fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    test) run pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    testx) run pytest_gpu 1200 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    bench) run bench 900 python bench.py --steps 30 --warmup 5 ;;
    benchfast) run bench 600 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    benchshard) run benchshard 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --sharded --steps 30 --warmup 5 --no-cpu-baseline ;;
    gemm) run gemm 300 python tools/gemm_bench.py ;;
    profshard) export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
      run profshard 900 rocprofv3 --kernel-trace --stats -T -d gpurun_out/profshard -o run --output-format csv -- python3 bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline --no-score
      unset MASTER_ADDR MASTER_PORT RANK LOCAL_RANK WORLD_SIZE ;;
    score) run score 600 python tools/score_bench.py ;;
    *) echo "unknown step $step" ;;
  esac
done
