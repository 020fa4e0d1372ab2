#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
step r3r_h 300 python3 -u tools/shard_host.py --steps 60
grep -v amdgpu.ids gpurun_out/r3r_h.log | grep "wall\|host\|  " | head -14
NCF_SHARD_OVERLAP_SWEEP=1 step r3r_hov 300 python3 -u tools/shard_host.py --steps 60
grep -v amdgpu.ids gpurun_out/r3r_hov.log | grep "wall\|host\|  " | head -14
