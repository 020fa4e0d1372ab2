# C2 step: the attention/tower fusion against the sweep / sort placements (A/B, interleaved)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5l}
timeout -k 10 600 python -u tools/step_ab.py --reps 3 unfused=engine.FUSE_ATTN_TOWER:0 \
  fused=engine.FUSE_ATTN_TOWER:1 \
  f_tower=engine.FUSE_ATTN_TOWER:1,env:NCF_SWEEP_FORK:tower \
  f_split=engine.FUSE_ATTN_TOWER:1,env:NCF_SWEEP_FORK:tower+mlp_bwd \
  f_sortemb=engine.FUSE_ATTN_TOWER:1,trainer.DEDUP_FORK:emb_bwd \
  f_sweep32=engine.FUSE_ATTN_TOWER:1,sweep:32 u_sweep32=engine.FUSE_ATTN_TOWER:0,sweep:32 \
  > gpurun_out/${T}_step_ab.log 2>&1
