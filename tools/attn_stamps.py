"""Per-phase time of the fused attention block kernels from in-kernel shader-clock stamps.

Needs a diagnostic build of the library (-DNCF_ATTN_STAMPS):
    NCF_OUT=abl/lib_astamps.so NCF_OBJ=/tmp/obj_ast NCF_EXTRA_FLAGS=-DNCF_ATTN_STAMPS ./build_ext.sh
    NCF_HIP_LIB=abl/lib_astamps.so python tools/attn_stamps.py
Runs C2 training steps (FusedTrainStep), then reads the stamps of the last forward and backward
(stashing forms): for each phase the mean over workgroups of (stamp[k+1] - stamp[k]) in shader
cycles."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402

ncf = _ncf_pkg.load()
FWD = ["stage x_u, x_i", "q/k/v projections", "tiles -> LDS", "stash q/k/v", "core",
       "stash o + out_proj + tiles", "y store"]
BWD = ["stage dY/q/k/v/o", "dO + out_proj dW", "core: dS, dQ", "core: dK, dV",
       "stash dq/dk/dv + q/k/v dW", "dX projections", "tiles -> LDS", "dX store"]


def main():
    from ncf_amd import _lib
    from ncf_amd.trainer import FusedTrainStep
    dev = torch.device("cuda", 0)
    D = int(os.environ.get("STAMP_D", "64"))
    U, I, B, M = 1_000_000, 100_000, 4096, 5
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, 32, [256, 128, 64], 4, 0.2, M - 1).to(dev).train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
    batches = bench.make_batches(U, I, B, M, 4, dev, seed=7)
    for s in range(8):
        step(*batches[s % 4])
    torch.cuda.synchronize()
    buf = np.zeros((2, 1024, 16), dtype=np.uint64)
    lib = _lib.load()
    rc = lib.ncf_debug_attn_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, "not a -DNCF_ATTN_STAMPS build?"
    nwg = min(1024, -(-B // (16 if D == 64 else 8)))
    for d, names in ((0, FWD), (1, BWD)):
        st = buf[d, :nwg, :len(names) + 1].astype(np.int64)
        dur = np.diff(st, axis=1)
        tot = st[:, -1] - st[:, 0]
        print(f"{'forward' if d == 0 else 'backward'} (D={D}): {nwg} workgroups, mean "
              f"{tot.mean():.0f} cycles per workgroup; start spread "
              f"{st[:, 0].max() - st[:, 0].min()} cycles, end spread {st[:, -1].max() - st[:, -1].min()}")
        for k, n in enumerate(names):
            print(f"  {n:26s} {dur[:, k].mean():9.0f} cycles  {100 * dur[:, k].mean() / tot.mean():5.1f}%"
                  f"  (min {dur[:, k].min()}, max {dur[:, k].max()})")


if __name__ == "__main__":
    main()
