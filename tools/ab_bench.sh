#!/bin/bash
# A/B: the C2 bench once per library build (NCF_HIP_LIB), twice each, interleaved.
#   bash tools/ab_bench.sh lib_a.so lib_b.so ...
mkdir -p gpurun_out
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    NCF_HIP_LIB="$L" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-score \
      > gpurun_out/ab_${n}_$rep.log 2>&1 || exit $?
    python3 - "$n" "$rep" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.log") if l.startswith("{")][-1])
k = d["kernel_ms_per_step"]
print(sys.argv[1], sys.argv[2], d["ms_per_step"], {x: k.get(x) for x in ("ncf_mlp_fwd", "ncf_mlp_bwd", "ncf_embedding_bwd_reduce", "ncf_reduce_batch", "ncf_attn_block_fwd", "ncf_attn_block_bwd")})
PY
  done
done
