"""Time the fused MLP tower kernels (GPU only) at C2 shape under variants:
train (saves r/a/mean/rstd) vs eval (no saves), dropout 0 vs 0.2.
    python tools/mlp_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402

ncf = _ncf_pkg.load()
from ncf_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = ncf.AdvancedNCF(100000, 100000, 10, 50).to(dev)
    eng = m.engine
    n = 20480
    g = torch.Generator(device=dev).manual_seed(1)
    u = torch.randint(0, 100000, (n,), generator=g, device=dev)
    i = torch.randint(0, 100000, (n,), generator=g, device=dev)
    for train, M in ((True, 5), (False, 1)):
        for p in (0.0, 0.2):
            if not train and p:
                continue
            for _ in range(3):
                eng.forward(u, i, M, train, p, 7)
            torch.cuda.synchronize()
            _lib.PROFILE = []
            for _ in range(20):
                eng.forward(u, i, M, train, p, 7)
            torch.cuda.synchronize()
            prof, _lib.PROFILE = _lib.PROFILE, None
            t = [e0.elapsed_time(e1) for name, _, e0, e1 in prof if name == "ncf_mlp_fwd"]
            t.sort()
            print(f"train={train} p={p}: ncf_mlp_fwd median {t[len(t) // 2] * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
