set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/dropin_host.py --warmup 5 --steps 60 > gpurun_out/r3b_host_early.log 2>&1 && \
timeout -k 10 200 python3 -u tools/dropin_host.py --warmup 200 --steps 200 --profile > gpurun_out/r3b_host_late.log 2>&1
echo rc=$?
