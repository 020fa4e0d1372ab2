#!/bin/bash
# Round-3: tower versions A/B (round-2 end b6cf6c4, C4 templating 1671527, HEAD), isolated k_mlp_bwd.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
B="python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4 --no-dropin"
K="ncf_mlp_bwd ncf_mlp_fwd"
for rep in 1 2; do
step r3ah_head_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ah_head_$rep.log $K
NCF_HIP_LIB=abl/lib_old.so step r3ah_r2_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ah_r2_$rep.log $K
NCF_HIP_LIB=abl/lib_mid.so step r3ah_mid_$rep 300 $B && python3 tools/bench_summ.py gpurun_out/r3ah_mid_$rep.log $K
done
