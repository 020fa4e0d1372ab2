"""Repeat the guarded fused step (tools/guard_bisect.py's run) K times in one process per mode
and report which repetitions differ from the first (GPU only): tells a result that depends on
what the memory held before (fixed by poisoning) from a cross-stream race (fixed by a fenced
event scope) from state left by an earlier run (fixed by collecting it between runs).

    python tools/repeat_diag.py [--k 5] [--fuse-apply 0] [--pipelined 0] MODE [MODE ...]
MODE: plain | noguard | poison | scope0 | scope1 | gc | nosmall | collect | alt | noguard_ec"""
import argparse
import contextlib
import gc
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import guard_bisect as GB  # noqa: E402
from ncf_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--fuse-apply", type=int, default=0)
    ap.add_argument("--early-reduce", type=int, default=0)
    ap.add_argument("--pipelined", type=int, default=0)
    ap.add_argument("modes", nargs="+")
    cfg = ap.parse_args()
    for mode in cfg.modes:
        scope0 = _lib.STREAM_EVENT_SCOPE
        small0 = _lib.query("ncf_dedup_set_small_max", -1)
        if mode == "scope0":
            _lib.STREAM_EVENT_SCOPE = 0
        if mode == "scope1":
            _lib.STREAM_EVENT_SCOPE = 1
        if mode == "nosmall":
            _lib.query("ncf_dedup_set_small_max", 0)
        if mode in ("noguard", "noguard_ec"):
            orig = GB.guarded
            GB.guarded = lambda poison=False, **kw: _NoGuard()
        res = []

        def collect(site):      # (per-allocation stack walk: slow host allocations, no poison)
            return False
        for r in range(cfg.k):
            slow = mode == "collect" or (mode == "alt" and r % 2 == 0)
            out = GB.run(cfg, collect if slow else mode == "poison")
            res.append(out)
            ok, bad, errs = GB.same(res[0], out)
            print(f"{mode} rep {r}: same_as_first {ok} err {out[2]} differ {len(bad)} {bad[:3]}",
                  flush=True)
            if mode in ("gc", "noguard_ec"):
                gc.collect()
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
            if mode == "noguard_ec":
                # a large allocation freed back to the driver between runs (test_gpu_c4's full-size
                # tables do this before the parity tests): the next run's segments may be handed
                # addresses that were mapped to other memory
                big = torch.empty(int(8e9), dtype=torch.uint8, device="cuda")
                big.fill_(7)
                del big
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
        _lib.STREAM_EVENT_SCOPE = scope0
        _lib.query("ncf_dedup_set_small_max", small0)
        if mode in ("noguard", "noguard_ec"):
            GB.guarded = orig


class _NoGuard(contextlib.AbstractContextManager):
    def __enter__(self):
        class A:
            @staticmethod
            def copy(t):
                return t.clone()
        return A()

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    main()
