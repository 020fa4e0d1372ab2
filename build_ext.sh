#!/bin/bash
# Build libncf_hip.so (gfx950) in-tree.  Used by __graft_entry__.build(); safe to run by hand.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")" && pwd)"
SRC="${NCF_SRC:-$ROOT/neural-collaborative-filtering-demo_amd/csrc}"   # NCF_SRC: A/B source trees
GEN="$ROOT/neural-collaborative-filtering-demo_amd/csrc/gen_fastcall.py"
OUT="${NCF_OUT:-$ROOT/neural-collaborative-filtering-demo_amd/libncf_hip.so}"   # NCF_OUT: A/B builds
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
OBJ="${NCF_OBJ:-$SRC/build}"
mkdir -p "$OBJ"
rm -f "$OBJ"/*.o
FLAGS=(--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$SRC" -I"$ROOT/include" -Wall -Wno-unused-function ${NCF_EXTRA_FLAGS:-})
# build identity compiled into capi.hip (ncf_build_info; checked by _lib.load())
ABI_HASH="$(python3 "$ROOT/neural-collaborative-filtering-demo_amd/_abi.py" abi)"
SRC_HASH="$(python3 "$ROOT/neural-collaborative-filtering-demo_amd/_abi.py" src "$SRC")"
NCF_FLAGS_capi="${NCF_FLAGS_capi:-} -DNCF_ABI_HASH=\"$ABI_HASH\" -DNCF_SRC_HASH=\"$SRC_HASH\""
pids=()
for f in "$SRC"/*.hip; do
  b="$(basename "$f" .hip)"
  per="NCF_FLAGS_$b"                     # per-file extra flags (A/B builds), e.g. NCF_FLAGS_adam
  "$HIPCC" "${FLAGS[@]}" ${!per:-} -c "$f" -o "$OBJ/$b.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" --offload-arch=gfx950 -shared -fPIC "$OBJ"/*.o -o "$OUT.tmp"
mv "$OUT.tmp" "$OUT"
echo "built $OUT"
# CPython fast-call binding of the C-ABI (generated from _lib.SIGNATURES; ctypes stays the
# loader and hands it the resolved entry points)
PYINC="$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')"
PYSUF="$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')"
python3 "$GEN" "$OBJ/_ncffast.c"
FAST="$(dirname "$OUT")/_ncffast$PYSUF"
gcc -O2 -shared -fPIC -I"$PYINC" "$OBJ/_ncffast.c" -o "$FAST.tmp"
mv "$FAST.tmp" "$FAST"
echo "built $FAST"
