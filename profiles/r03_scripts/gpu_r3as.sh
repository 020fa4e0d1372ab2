#!/bin/bash
# Round-3: two-pass attention core (softmax lanes, then float4 O over all threads) vs one lane
# per (group, head, query row): the full GPU suite, then an interleaved step A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3as_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3as_tests.log
step r3as_ab 600 bash tools/ab_libs.sh abl/lib_old.so abl/lib_new.so abl/lib_old.so abl/lib_new.so
python3 -c "
import json
for l in open('gpurun_out/r3as_ab.log'):
    d = json.loads(l); u = d['us']
    print(d['tag'], d['ms_per_step'], 'attn_fwd', u.get('ncf_attn_block_fwd'), 'attn_bwd', u.get('ncf_attn_block_bwd'), 'mlp_bwd', u.get('ncf_mlp_bwd'), 'loss', d['loss'])
"
