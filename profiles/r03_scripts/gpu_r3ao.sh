#!/bin/bash
# Round-3: layer-1 pre-LN rows kept in LDS through the tower backward (stash) vs read twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3ao_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -k "tower or train or golden or determin or bf16" -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/r3ao_tests.log
step r3ao_ab 600 bash tools/ab_libs.sh abl/lib_nostash.so abl/lib_stash.so abl/lib_nostash.so abl/lib_stash.so
python3 -c "
import json
for l in open('gpurun_out/r3ao_ab.log'):
    d = json.loads(l); u = d['us']
    print(d['tag'], d['ms_per_step'], 'mlp_bwd', u.get('ncf_mlp_bwd'), 'loss', d['loss'])
"
