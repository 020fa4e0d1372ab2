# round-5 evidence: full-size parity first, then the GPU suite, the driver's bench command,
# staging-batch stamps variants
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5g}
bash tools/gpu_run.sh $T t:fused_forward fullsize tests &&
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/tower_ab.py > gpurun_out/${T}_tower_ab.log 2>&1 &&
for sb in "" _sb5 _sb10; do
  NCF_HIP_LIB=build_alt/lib_stamps$sb.so timeout -k 10 300 python -u tools/mlp_stamps.py > gpurun_out/${T}_stamps$sb.log 2>&1 || exit $?
done
