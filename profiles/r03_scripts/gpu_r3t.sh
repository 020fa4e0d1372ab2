#!/bin/bash
# Round-3: attention block with 8 interaction groups per workgroup at D=64 (2 workgroups per CU).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'attn', k.get('ncf_attn_block_fwd'), k.get('ncf_attn_block_bwd'))"; }
NCF_HIP_LIB=abl/lib_g8.so step r3t_g8_tests 300 python3 -u -m pytest tests/test_gpu_parity.py -k "attn" -x -q --timeout 200 --timeout-method thread
tail -2 gpurun_out/r3t_g8_tests.log
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4 --no-dropin"
step r3t_def1 300 $B && summ r3t_def1
NCF_HIP_LIB=abl/lib_g8.so step r3t_g8_1 300 $B && summ r3t_g8_1
step r3t_def2 300 $B && summ r3t_def2
NCF_HIP_LIB=abl/lib_g8.so step r3t_g8_2 300 $B && summ r3t_g8_2
