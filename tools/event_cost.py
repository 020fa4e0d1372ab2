"""What a cross-stream fork / join costs the stream that carries the step (GPU only).
Between two kernels on the main stream, per iteration: nothing; an event record (the fork
point's marker); a record + a side-stream wait (a fork); a wait on a side-stream event that is
long complete; a full fork + side kernel + join.  The kernels are ~17 us (64 MB in-place adds),
so the loop is GPU-bound and the differences are queue time.
    python tools/event_cost.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402

_ncf_pkg.load()
from ncf_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    x = torch.zeros(16 << 20, device=dev)
    y = torch.zeros(1 << 20, device=dev)
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    ms, ss = main_s.cuda_stream, side.cuda_stream
    ev = [_lib.RawEvent(stream_only=True) for _ in range(4)]
    ev[3].record(ss)

    def it(mode):
        x.add_(1.0)
        if mode == "record":
            ev[0].record(ms)
        elif mode == "fork":
            ev[0].record(ms)
            ev[0].wait(ss)
        elif mode == "wait_done":
            ev[3].wait(ms)
        elif mode == "fork_join":
            ev[0].record(ms)
            ev[0].wait(ss)
            with torch.cuda.stream(side):
                y.add_(1.0)
            ev[1].record(ss)
            ev[1].wait(ms)
        x.add_(1.0)

    modes = ["plain", "record", "fork", "wait_done", "fork_join"]
    res = {m: [] for m in modes}
    for rep in range(4):
        for m in modes:
            for _ in range(50):
                it(m)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 2000
            for _ in range(n):
                it(m)
            torch.cuda.synchronize()
            res[m].append((time.perf_counter() - t0) / n * 1e6)
    base = min(res["plain"])
    for m in modes:
        v = min(res[m])
        print(f"{m:10s} {v:7.2f} us/iter  (+{v - base:5.2f})  runs {' '.join(f'{a:.2f}' for a in res[m])}",
              flush=True)


if __name__ == "__main__":
    main()
