# the register-only first reject of the scan (NCF_SCAN_MINTH): the C5 tests, then graphed C5
# against the same sources built with NCF_SCAN_MINTH=0 (ab_lib/libncf_hip_old.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5zi}
bash tools/gpu_run.sh $T "t:sample or score or topk or scan" || exit $?
for rep in 1 2; do
  for lib in ab_lib/libncf_hip_old.so neural-collaborative-filtering-demo_amd/libncf_hip.so; do
    echo "--- $lib ($rep)" >> gpurun_out/${T}_c5.log
    NCF_HIP_LIB=$lib timeout -k 10 200 python -u tools/score_bench.py --graph --reps 3 \
      >> gpurun_out/${T}_c5.log 2>&1 || exit $?
  done
done
