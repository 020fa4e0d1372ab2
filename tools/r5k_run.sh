# kernel timelines of the C2 step with the attention/tower fusion on and off (early catch-up off)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5k}
for v in fused=engine.FUSE_ATTN_TOWER:1,deferred.EARLY_CATCHUP:0 unfused=engine.FUSE_ATTN_TOWER:0,deferred.EARLY_CATCHUP:0; do
  n=${v%%=*}
  rm -rf gpurun_out/${T}_tl_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tl_$n -o run -- \
    python3 tools/step_ab.py --reps 1 --steps 60 $v > gpurun_out/${T}_tl_$n.log 2>&1 || exit $?
done
