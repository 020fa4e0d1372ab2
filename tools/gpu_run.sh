#!/bin/bash
# One GPU-box session: tools/gpu_run.sh TAG STEP [STEP ...], run from the repo root by gpurun.
# Steps (each under its own time limit; the first failure ends the run):
#   tests            the whole -m gpu suite
#   fullsize         tests/test_gpu_fullsize.py only
#   t:<pytest -k>    the -m gpu tests matching the expression
#   bench            python bench.py (defaults), JSON line -> gpurun_out/TAG_bench.json
#   quick            bench.py --steps 100 --warmup 10 --no-c4 --no-score
#   sharded          bench.py --sharded (the row-sharded step at world 1) -> TAG_sharded.json
#   dropinhost       tools/dropin_host.py (host time of the reference call pattern, cProfile)
#   prof             rocprofv3 --kernel-trace --stats over a short bench (C2 legs only)
#   pmc              FETCH_SIZE / WRITE_SIZE passes over the same command (tools/pmc_run.sh;
#                    -> profiles/TAG_pmc_traffic.json, copied to gpurun_out/)
#   dropinprof       rocprofv3 --kernel-trace --stats over tools/dropin_host.py (gaps per phase)
#   c5pmc            FETCH_SIZE / WRITE_SIZE passes over tools/score_bench.py (-> TAG_c5_pmc_traffic.json)
#   c5sq             SQ counters (tools/pmc_sq.sh, 3 passes) over tools/score_bench.py --k 10
#   c5prof           rocprofv3 --kernel-trace --stats over tools/score_bench.py
#   ab:VAR=a,b       the short C2 bench with VAR=a and VAR=b, interleaved 3 times each
#                    (ms/step + the per-kernel ms of each run -> TAG_ab.log)
#   sab:VAR=a,b      the row-sharded bench at world 1 (torchrun, 1 rank) with VAR=a / VAR=b, twice
#   c5ab:VAR=a,b     tools/score_bench.py (10K users x 1M items, top-10 / top-100, eager, per-stage
#                    ms) with VAR=a and VAR=b, interleaved twice each -> TAG_c5ab.log
# Output: gpurun_out/TAG_<step>.log (+ .json / prof dirs).
set -o pipefail
TAG=$1
shift
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
md5sum neural-collaborative-filtering-demo_amd/*.so > "$OUT/${TAG}_so.md5" 2>/dev/null
# the build identity compiled into the library next to the hashes of this tree (_abi.py)
python3 - >> "$OUT/${TAG}_so.md5" 2>&1 <<'PYEOF'
import ctypes, subprocess
lib = ctypes.CDLL("neural-collaborative-filtering-demo_amd/libncf_hip.so")
lib.ncf_build_info.restype = ctypes.c_char_p
tree = [subprocess.run(["python3", "neural-collaborative-filtering-demo_amd/_abi.py", k],
                       capture_output=True, text=True).stdout.strip() for k in ("abi", "src")]
print("library:", lib.ncf_build_info().decode(), "| tree: abi=%s src=%s" % tuple(tree))
PYEOF
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
QUICK="bench.py --steps 60 --warmup 10 --prime 128 --no-c4 --no-score --no-cpu-baseline --no-dropin --no-extra"
for what in "$@"; do
  echo "== $TAG $what $(date +%T)"
  case "$what" in
    tests)
      timeout -k 10 1100 $PYT tests -m gpu > "$OUT/${TAG}_tests.log" 2>&1
      rc=$? ;;
    fullsize)
      timeout -k 10 600 $PYT -v tests/test_gpu_fullsize.py > "$OUT/${TAG}_fullsize.log" 2>&1
      rc=$? ;;
    t:*)
      timeout -k 10 600 $PYT -v tests -m gpu -k "${what#t:}" > "$OUT/${TAG}_t.log" 2>&1
      rc=$? ;;
    bench)
      timeout -k 10 900 python -u bench.py > "$OUT/${TAG}_bench.log" 2>&1
      rc=$?
      grep '^{' "$OUT/${TAG}_bench.log" | tail -1 > "$OUT/${TAG}_bench.json" ;;
    quick)
      timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-c4 --no-score --no-extra \
        > "$OUT/${TAG}_quick.log" 2>&1
      rc=$?
      grep '^{' "$OUT/${TAG}_quick.log" | tail -1 > "$OUT/${TAG}_quick.json" ;;
    sharded)
      timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --sharded --steps 200 --warmup 20 \
        --no-c4 --no-score --no-cpu-baseline --no-dropin > "$OUT/${TAG}_sharded.log" 2>&1
      rc=$?
      grep '^{' "$OUT/${TAG}_sharded.log" | tail -1 > "$OUT/${TAG}_sharded.json" ;;
    dropinhost)
      timeout -k 10 300 python -u tools/dropin_host.py > "$OUT/${TAG}_dropinhost.log" 2>&1
      rc=$? ;;
    prof)
      rm -rf "$OUT/${TAG}_prof"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- \
        python3 $QUICK > "$OUT/${TAG}_prof.log" 2>&1
      rc=$? ;;
    pmc)
      PMC_CMD="python3 $QUICK" timeout -k 10 700 bash tools/pmc_run.sh "$TAG" \
        > "$OUT/${TAG}_pmc.log" 2>&1
      rc=$?
      cp "profiles/${TAG}_pmc_traffic.json" "$OUT/" 2>/dev/null ;;
    dropinprof)
      rm -rf "$OUT/${TAG}_dropinprof"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_dropinprof" -o run -- \
        python3 tools/dropin_host.py --warmup 150 --steps 60 > "$OUT/${TAG}_dropinprof.log" 2>&1
      rc=$? ;;
    c5pmc)
      PMC_CMD="python3 tools/score_bench.py --k 10 100 --reps 1" timeout -k 10 500 \
        bash tools/pmc_run.sh "${TAG}_c5" > "$OUT/${TAG}_c5pmc.log" 2>&1
      rc=$?
      cp "profiles/${TAG}_c5_pmc_traffic.json" "$OUT/" 2>/dev/null ;;
    c5sq)
      SQ_CMD="python3 tools/score_bench.py --k 10 --reps 1" timeout -k 10 500 \
        bash tools/pmc_sq.sh "${TAG}c5" > "$OUT/${TAG}_c5sq.log" 2>&1
      rc=$?
      python3 tools/pmc_sq_summary.py "${TAG}c5" collect,sample,kth,select >> "$OUT/${TAG}_c5sq.log" 2>&1 ;;
    c5prof)
      rm -rf "$OUT/${TAG}_c5prof"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c5prof" -o run -- \
        python3 tools/score_bench.py > "$OUT/${TAG}_c5prof.log" 2>&1
      rc=$? ;;
    ab:*)
      spec="${what#ab:}"; var="${spec%%=*}"; vals="${spec#*=}"; va="${vals%%,*}"; vb="${vals#*,}"
      rc=0
      for k in 1 2 3; do
        for v in "$va" "$vb"; do
          f="$OUT/${TAG}_ab_$(basename "$v")_$k.log"
          env "$var=$v" timeout -k 10 200 python3 $QUICK > "$f" 2>&1 || { rc=$?; break 2; }
          python3 tools/bench_summ.py "$f" "$var=$v" >> "$OUT/${TAG}_ab.log" 2>&1
        done
      done ;;
    sab:*)
      spec="${what#sab:}"; var="${spec%%=*}"; vals="${spec#*=}"; va="${vals%%,*}"; vb="${vals#*,}"
      rc=0
      for k in 1 2; do
        for v in "$va" "$vb"; do
          f="$OUT/${TAG}_sab_$(basename "$v")_$k.log"
          env "$var=$v" timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --sharded \
            --steps 100 --warmup 20 --prime 128 --no-c4 --no-score --no-cpu-baseline --no-dropin \
            > "$f" 2>&1 || { rc=$?; break 2; }
          python3 tools/bench_summ.py "$f" "$var=$v" >> "$OUT/${TAG}_sab.log" 2>&1
        done
      done ;;
    dirsab:*)
      # dirsab:DIR  the row-sharded bench at world 1 from DIR (another checkout, e.g. a git
      # worktree of an earlier commit with its own built libraries) and from here, alternately
      d="${what#dirsab:}"
      rc=0
      for k in 1 2; do
        for where in "$d" .; do
          f="$OUT/${TAG}_dirsab_$(basename "$where")_$k.log"
          extra=""
          [ "$where" = "." ] && extra="--batches 8"   # (the earlier bench cycled 8 batches)
          (cd "$where" && timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --sharded \
            --steps 100 --warmup 20 --prime 128 --no-c4 --no-score --no-cpu-baseline \
            --no-dropin $extra) > "$f" 2>&1 || { rc=$?; break 2; }
          python3 tools/bench_summ.py "$f" "dir=$where" >> "$OUT/${TAG}_dirsab.log" 2>&1
        done
      done ;;
    c5ab:*)
      spec="${what#c5ab:}"; var="${spec%%=*}"; vals="${spec#*=}"; va="${vals%%,*}"; vb="${vals#*,}"
      rc=0
      for k in 1 2; do
        for v in "$va" "$vb"; do
          echo "--- $var=$v ($k)" >> "$OUT/${TAG}_c5ab.log"
          env "$var=$v" timeout -k 10 200 python3 tools/score_bench.py >> "$OUT/${TAG}_c5ab.log" 2>&1 || { rc=$?; break 2; }
        done
      done ;;
    *)
      echo "unknown step $what"; exit 2 ;;
  esac
  # a GPU fault in any log of this step ends the session (exit 99): nothing more runs on the card
  if grep -qsE "illegal memory access|Memory access fault|GPU fault|hipErrorLaunchFailure|HSA_STATUS_ERROR" \
      "$OUT/${TAG}_"*"${what%%:*}"*.log; then
    echo "== $TAG $what: GPU fault in the log, stopping"
    rc=99
  fi
  echo "== $TAG $what rc=$rc $(date +%T)"
  if [ $rc -ne 0 ]; then
    tail -40 "$OUT/${TAG}_"*"${what%%:*}"*.log 2>/dev/null
    exit $rc
  fi
done
