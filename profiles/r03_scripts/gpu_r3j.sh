#!/bin/bash
# Round-3 A/B: the piece-reduce grid cap (NCF_PIECE_BLOCKS_MAX builds in abl/), C2 bench only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
summ() { python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/$1.log') if l.startswith('{')][-1]; k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], 'emb', k.get('ncf_embedding_bwd_reduce'), 'red', k.get('ncf_reduce_batch'), 'dropin', d['dropin_train']['ms_per_step'])"; }
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
step r3j_def 400 $B && summ r3j_def
for b in 128 256 512; do
  NCF_HIP_LIB=abl/lib_pb$b.so step r3j_pb$b 400 $B && summ r3j_pb$b
done
step r3j_def2 400 $B && summ r3j_def2
