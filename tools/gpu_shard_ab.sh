# sharded world-1 step: the overlapped sweep at several fork points (bench --sharded)
set -o pipefail
mkdir -p gpurun_out
i=0
for cfg in off mlp_bwd tower reduce attn_bwd; do
  i=$((i+1))
  if [ $cfg = off ]; then o=0; f=mlp_bwd; else o=1; f=$cfg; fi
  NCF_SHARD_OVERLAP_SWEEP=$o NCF_SWEEP_FORK=$f MASTER_ADDR=127.0.0.1 MASTER_PORT=2954$i RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 \
    timeout -k 10 300 python -u bench.py --sharded --steps 200 --warmup 140 --no-cpu-baseline --no-score --no-c4 > gpurun_out/sh_ab_$cfg.log 2>&1 || exit 1
  grep '^{' gpurun_out/sh_ab_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded $cfg', d['ms_per_step'])"
done
