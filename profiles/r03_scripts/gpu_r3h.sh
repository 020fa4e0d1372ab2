#!/bin/bash
# Round-3: GPU suite (shared-Q parity), then A/B: default / claim off / shared Q off, and stamps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'attn', k.get('ncf_attn_block_fwd'), k.get('ncf_attn_block_bwd'), 'dropin', d['dropin_train']['ms_per_step'], d['dropin_train']['with_loss_item']['ms_per_step'])"; }
step r3h_tests 900 python3 -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread
grep -E "shared Q|passed|failed" gpurun_out/r3h_tests.log | tail -8
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
step r3h_bench_def 400 $B && summ r3h_bench_def
NCF_CLAIM_CATCHUP=0 step r3h_bench_noclaim 400 $B && summ r3h_bench_noclaim
NCF_ATTN_SHARE_Q=0 step r3h_bench_noshq 400 $B && summ r3h_bench_noshq
NCF_HIP_LIB=abl/lib_astamps.so step r3h_attn_stamps 200 python3 -u tools/attn_stamps.py
grep -v amdgpu.ids gpurun_out/r3h_attn_stamps.log
step r3h_dropin_host 300 python3 -u tools/dropin_host.py --warmup 150 --steps 100
head -45 gpurun_out/r3h_dropin_host.log | grep -v amdgpu.ids
