#!/bin/bash
# Round-3: suite; attention stamps (shared Q on/off); bench (C2 + C5, grouped candidate flush);
# C5 scan PMC write traffic.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3k_tests 900 python3 -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread
grep -E "shared Q|passed|failed" gpurun_out/r3k_tests.log | tail -7
NCF_HIP_LIB=abl/lib_astamps.so step r3k_stamps_shq 200 python3 -u tools/attn_stamps.py
grep -v amdgpu.ids gpurun_out/r3k_stamps_shq.log | head -9
NCF_ATTN_SHARE_Q=0 NCF_HIP_LIB=abl/lib_astamps.so step r3k_stamps_noshq 200 python3 -u tools/attn_stamps.py
grep -v amdgpu.ids gpurun_out/r3k_stamps_noshq.log | head -9
step r3k_bench 600 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c4
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r3k_bench.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; c=d['c5_scoring']; print('C2', d['ms_per_step'], 'attn', k.get('ncf_attn_block_fwd'), k.get('ncf_attn_block_bwd'), 'dropin', d['dropin_train']['ms_per_step']); print('C5', c['item_index_ms'], c['k10']['ms'], c['k10']['collect_ms'], c['k100']['ms'], c['k100']['collect_ms'])"
for C in FETCH_SIZE WRITE_SIZE; do
  step r3k_pmc_$C 200 rocprofv3 --pmc $C -d gpurun_out/r3k_pmc_$C -o run --output-format csv -- python3 tools/score_bench.py --reps 1
done
python3 tools/pmc_traffic.py gpurun_out/r3k_pmc_FETCH_SIZE gpurun_out/r3k_pmc_WRITE_SIZE gpurun_out/r3k_c5_pmc_traffic.json && grep -A3 collect3 gpurun_out/r3k_c5_pmc_traffic.json | head -12
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'emb', k.get('ncf_embedding_bwd_reduce'), 'red', k.get('ncf_reduce_batch'), 'dropin', d['dropin_train']['ms_per_step'])"; }
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
step r3k_def 400 $B && summ r3k_def
NCF_HIP_LIB=abl/lib_pb256.so step r3k_pb256 400 $B && summ r3k_pb256
