#!/bin/bash
# Round-3: world-1 sharded step A/B, interleaved and repeated on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
B="python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
show() { grep '^{' gpurun_out/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'])"; }
p=29570
for rep in 1 2; do
  for cfg in def ov a0 a0ov; do
    p=$((p+1))
    case $cfg in
      def) E="";; ov) E="NCF_SHARD_OVERLAP_SWEEP=1";; a0) E="NCF_SHARD_AHEAD=0";; a0ov) E="NCF_SHARD_AHEAD=0 NCF_SHARD_OVERLAP_SWEEP=1";;
    esac
    env_cmd="MASTER_PORT=$p $E"
    eval "export $env_cmd"
    step r3s_${cfg}_$rep 300 $B && show r3s_${cfg}_$rep
    unset NCF_SHARD_AHEAD NCF_SHARD_OVERLAP_SWEEP
  done
done
