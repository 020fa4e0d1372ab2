# fused attention/tower (attention weight prefetch off: 196 VGPRs) vs unfused, sweep placements
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5m}
bash tools/gpu_run.sh $T "t:attn_tower_fused" || exit $?
timeout -k 10 600 python -u tools/step_ab.py --reps 3 unfused=engine.FUSE_ATTN_TOWER:0 \
  fused=engine.FUSE_ATTN_TOWER:1 \
  f_tower=engine.FUSE_ATTN_TOWER:1,env:NCF_SWEEP_FORK:tower \
  u_tower=engine.FUSE_ATTN_TOWER:0,env:NCF_SWEEP_FORK:tower \
  > gpurun_out/${T}_step_ab.log 2>&1 || exit $?
bash tools/gpu_run.sh $T fullsize
