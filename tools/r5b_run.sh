# round-5 session-1 evidence: GPU suite, the driver's bench command, isolated tower times,
# tower phase stamps (diagnostic build in build_alt/)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_run.sh r5b tests &&
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5b_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/tower_ab.py > gpurun_out/r5b_tower_ab.log 2>&1 &&
NCF_HIP_LIB=build_alt/lib_stamps.so timeout -k 10 300 python -u tools/mlp_stamps.py > gpurun_out/r5b_stamps.log 2>&1
