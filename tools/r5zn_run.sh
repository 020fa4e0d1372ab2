# the row-sharded step at world 1: rolling-sweep period 64 / 128 (distributed.SWEEP_EVERY)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zn}
for rep in 1 2; do
  for v in 64 128; do
    f=gpurun_out/${T}_sab_${v}_${rep}.log
    timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29521 tools/bench_set.py --set distributed.SWEEP_EVERY=$v \
      -- --sharded --steps 200 --warmup 20 --no-c4 --no-score --no-cpu-baseline --no-dropin \
      > $f 2>&1 || exit $?
    echo "SWEEP_EVERY=$v ($rep): $(grep '^{' $f | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" >> gpurun_out/${T}_sab.log
  done
done
