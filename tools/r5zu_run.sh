# the fused apply as a template argument (the reduce without it back to its own register budget):
# the bitwise / bf16 / sharded tests, then the fused and the world-1 sharded step against the HEAD
# library (ab_lib/libncf_hip_old.so), alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zu}
bash tools/gpu_run.sh $T "t:fused_apply or late_catchup or deferred or bitwise or bf16 or sharded" || exit $?
for rep in 1 2; do
  for lib in ab_lib/libncf_hip_old.so neural-collaborative-filtering-demo_amd/libncf_hip.so; do
    echo "--- $lib ($rep)" >> gpurun_out/${T}_ab.log
    NCF_HIP_LIB=$lib timeout -k 10 300 python -u tools/step_ab.py --reps 1 base=trainer.FUSE_APPLY:1 \
      >> gpurun_out/${T}_ab.log 2>&1 || exit $?
    f=gpurun_out/${T}_sab_$(basename $lib)_$rep.log
    NCF_HIP_LIB=$lib timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29523 bench.py --sharded --steps 200 --warmup 20 \
      --no-c4 --no-score --no-cpu-baseline --no-dropin > $f 2>&1 || exit $?
    echo "sharded $(grep '^{' $f | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> gpurun_out/${T}_ab.log
  done
done
