for rep in 1 2; do for A in 0 1; do
NCF_SHARD_AHEAD=$A timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2955$A bench.py --sharded --steps 40 --warmup 5 --no-cpu-baseline --no-score > gpurun_out/abs_${A}_$rep.log 2>&1 || exit $?
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abs_${A}_$rep.log') if l.startswith('{')][-1]); print('ahead=$A rep $rep', d['ms_per_step'])"
done; done
