#!/usr/bin/env python3
"""VALU issue slots per element-step of the deferred-Adam replay loops, from the gfx950 ISA.

    python tools/isa_replay_count.py [adam.s]      # (hipcc --cuda-device-only -S csrc/adam.hip)

For each kernel whose symbol matches (the rolling sweep k_pairs_sweep, the catch-ups
k_pairs_catchup / k_pairs_catchup_claim, D = 64 and 128, fp32 tables) it finds the innermost
loop holding the most v_sqrt_f32 (the replay's chunk loop: one sqrt per element-step, adam0 in
csrc/adam.hip) and counts its vector instructions.  Issue slots: a wave64 VALU instruction
occupies its SIMD 2 cycles (32 lanes / cycle), a packed one (v_pk_fma_f32 / v_pk_mul_f32: two
fp32 ops per lane) counts 2 slots, a transcendental one (v_sqrt / v_rcp / v_exp / v_log / v_rsq)
8 cycles (quarter rate; MI355X_MICROARCH.md 'vector-instruction ISSUE cost'): 4 slots.  bench.py prices the table Adam against the chip's VALU issue
rate with these numbers (ADAM_REPLAY_ISA); this script regenerates them.
"""
import json
import re
import subprocess
import sys

TRANS = ("v_sqrt_", "v_rcp_", "v_exp_", "v_log_", "v_rsq_", "v_sin_", "v_cos_")


def kernels(asm):
    cur, out = None, {}
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                cur = None
                continue
            out[cur].append(line.strip())
    return out


def loops(body):
    """(start, end) index spans of backward branches."""
    labels = {}
    spans = []
    for k, ln in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            labels[m.group(1)] = k
        m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)", ln)
        if m and m.group(2) in labels:
            spans.append((labels[m.group(2)], k))
    return spans


def count(lines):
    c = {"valu": 0, "packed": 0, "trans": 0, "salu": 0, "smem": 0, "vmem": 0, "sqrt": 0}
    for ln in lines:
        op = ln.split()[0] if ln and not ln.startswith((";", ".")) else ""
        if op.startswith("v_"):
            if op.startswith(TRANS):
                c["trans"] += 1
            elif op.startswith("v_pk_"):
                c["packed"] += 1
            else:
                c["valu"] += 1
            if op.startswith("v_sqrt_"):
                c["sqrt"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            c["smem"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("s_") and not op.startswith(("s_waitcnt", "s_nop")):
            c["salu"] += 1
    return c


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else None
    if src is None:
        src = "/tmp/adam_isa.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-Ineural-collaborative-filtering-demo_amd/csrc", "-Iinclude",
                        "--cuda-device-only", "-S",
                        "neural-collaborative-filtering-demo_amd/csrc/adam.hip", "-o", src],
                       check=True)
    asm = open(src).read()
    res = {}
    for sym, body in kernels(asm).items():
        m = re.search(r"k_pairs_(sweep|catchup_claim|catchup)ILi(64|128)ELb0E", sym)
        if not m:
            continue
        best = None
        sp = loops(body)
        for a, b in sp:
            if any(a <= a2 and b2 <= b and (a2, b2) != (a, b) and count(body[a2:b2 + 1])["sqrt"]
                   for a2, b2 in sp):
                continue          # not innermost: a replay loop nests inside it
            c = count(body[a:b + 1])
            if c["sqrt"] and (best is None or c["sqrt"] > best["sqrt"]
                              or (c["sqrt"] == best["sqrt"] and b - a < best["len"])):
                best = dict(c, len=b - a)
        if best is None:
            continue
        es = best["sqrt"]
        res[f"{m.group(1)}_D{m.group(2)}"] = {
            "element_steps_per_iteration": es,
            "valu_per_element_step": round(best["valu"] / es, 3),
            "packed_per_element_step": round(best["packed"] / es, 3),
            "transcendental_per_element_step": round(best["trans"] / es, 3),
            "issue_slots_per_element_step": round(
                (best["valu"] + 2 * best["packed"] + 4 * best["trans"]) / es, 3),
            "salu_smem_per_iteration": best["salu"] + best["smem"]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
