# the drop-in optimiser's rolling-sweep period (optim.SWEEP_EVERY 64 / 128): the reference-loop leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zq}
for rep in 1 2; do
  for v in 64 128; do
    f=gpurun_out/${T}_dropin_${v}_${rep}.log
    timeout -k 10 300 python3 tools/bench_set.py --set optim.SWEEP_EVERY=$v -- --steps 200 \
      --no-c4 --no-score --no-extra --no-cpu-baseline > $f 2>&1 || exit $?
    echo "SWEEP_EVERY=$v ($rep): $(grep '^{' $f | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["dropin_train"]["ms_per_step"], d["ms_per_step"])')" >> gpurun_out/${T}_dropin.log
  done
done
