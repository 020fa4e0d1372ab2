#!/bin/bash
# Round-3: position-ordered embedding backward (focused parity first), then the suite and A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3g_focus 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -k "position_reduce or segment_reduce or bf16_deferred_bitwise" -x -v -s --timeout 200 --timeout-method thread
grep -E "passed|failed|pos vs piece" gpurun_out/r3g_focus.log | tail -9
step r3g_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -2 gpurun_out/r3g_tests.log
for pos in 0 1; do
  NCF_EMB_POS=$pos step r3g_bench_pos$pos 400 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r3g_bench_pos$pos.log') if l.startswith('{')][-1]; print('pos=$pos', d['ms_per_step'], d['kernel_ms_per_step'].get('ncf_embedding_bwd_reduce'), 'dropin', d['dropin_train']['ms_per_step'])"
done
for cl in 0 1; do
  NCF_CLAIM_CATCHUP=$cl step r3g_dropin_claim$cl 300 python3 -u tools/dropin_probe.py --trace 12 --windows 3
  tail -1 gpurun_out/r3g_dropin_claim$cl.log | cut -c1-700
done
NCF_HIP_LIB=abl/lib_astamps.so step r3g_attn_stamps 200 python3 -u tools/attn_stamps.py
cat gpurun_out/r3g_attn_stamps.log | grep -v amdgpu.ids
