# session check: tests, bench (no C4/CPU), early-catch-up A/B, sharded world-1 with/without the overlapped sweep
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_quick.sh || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/q_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']); print(d['kernel_ms_per_step']); print('dropin', d['dropin_train']['ms_per_step'], 'bf16', d['c2_bf16_tables']['ms_per_step'])"
for e in 0 1; do
  NCF_EARLY_CATCHUP=$e timeout -k 10 120 python -u tools/kernel_ab.py --tag early$e 2>&1 | grep '^{' || exit 1
done
for o in 0 1; do
  NCF_SHARD_OVERLAP_SWEEP=$o MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$o RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 timeout -k 10 300 python -u bench.py --sharded --steps 200 --warmup 140 --no-cpu-baseline --no-score --no-c4 > gpurun_out/sh_bench$o.log 2>&1 || exit 1
  grep '^{' gpurun_out/sh_bench$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded overlap=$o', d['ms_per_step'])"
done
