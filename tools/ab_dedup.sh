#!/bin/bash
# A/B the dedup (radix digit width builds): C2 bench twice per library, interleaved; prints the
# step time and the dedup / embedding-backward launch times.
mkdir -p gpurun_out
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    NCF_HIP_LIB="$L" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-score \
      > gpurun_out/abd_${n}_$rep.log 2>&1 || exit $?
    python3 - "$n" "$rep" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/abd_{sys.argv[1]}_{sys.argv[2]}.log") if l.startswith("{")][-1])
k = d["kernel_ms_per_step"]
print(sys.argv[1], sys.argv[2], d["ms_per_step"], {x: k.get(x) for x in ("ncf_dedup_ids", "ncf_embedding_bwd_reduce")})
PY
  done
done
