"""Per-phase time of the fused MLP tower kernels from in-kernel shader-clock stamps.

Needs a diagnostic build of the library (-DNCF_MLP_STAMPS):
    NCF_OUT=abl/lib_stamps.so NCF_OBJ=/tmp/obj_st NCF_EXTRA_FLAGS=-DNCF_MLP_STAMPS ./build_ext.sh
    NCF_HIP_LIB=abl/lib_stamps.so python tools/mlp_stamps.py
Runs C2 training steps (FusedTrainStep), then reads the stamps of the last forward and backward:
for each phase the mean over workgroups of (stamp[k+1] - stamp[k]) in shader cycles, and the
spread of the workgroups' start and end times."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402
import bench  # noqa: E402

ncf = _ncf_pkg.load()
FWD = ["stage x", "lin0 (64->256)", "ln0", "lin1 (256->128)", "ln1", "lin2 (128->64)",
       "ln2 + head"]
FWD_PIPE = ["stage x", "lin0 A", "lin0 B | ln0 A", "lin1 A | ln0 B", "lin1 B | ln1 A",
            "lin2 A | ln1 B", "lin2 B | ln2 A", "ln2 B + head"]
BWD = ["head bwd", "ln2 bwd", "stage a1", "wgrad2", "lin2 bwd", "ln1 bwd", "stage a0", "wgrad1",
       "lin1 bwd", "ln0 bwd", "stage x", "wgrad0", "lin0 bwd", "dx store"]


def main():
    import ncf_amd.engine as E
    from ncf_amd import _lib
    from ncf_amd.trainer import FusedTrainStep
    # --fp32: the tower on fp32 MFMA (engine.TOWER_SPLIT off); default: the engine's setting
    if "--fp32" in sys.argv:
        E.TOWER_SPLIT = False
    print(f"tower split operands: {E.TOWER_SPLIT}")
    dev = torch.device("cuda", 0)
    U, I, B, M = 1_000_000, 100_000, 4096, 5
    m = ncf.AdvancedNCF(U, I, 10, 50, 64, 64, 32, [256, 128, 64], 4, 0.2, M - 1).to(dev).train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
    batches = bench.make_batches(U, I, B, M, 4, dev, seed=7)
    for s in range(8):
        step(*batches[s % 4])
    torch.cuda.synchronize()
    buf = np.zeros((2, 1024, 16), dtype=np.uint64)
    lib = _lib.load()
    rc = lib.ncf_debug_mlp_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, "not a -DNCF_MLP_STAMPS build?"
    nwg = (B * M + 79) // 80
    fwd = FWD_PIPE if buf[0, 0, 8] != 0 else FWD   # the pipelined forward stamps 9 points
    for d, names in ((0, fwd), (1, BWD)):
        st = buf[d, :nwg, :len(names) + 1].astype(np.int64)
        dur = np.diff(st, axis=1)
        tot = st[:, -1] - st[:, 0]
        print(f"{'forward' if d == 0 else 'backward'}: {nwg} workgroups, mean {tot.mean():.0f} "
              f"cycles per workgroup; start spread {st[:, 0].max() - st[:, 0].min()} cycles, "
              f"end spread {st[:, -1].max() - st[:, -1].min()}")
        for k, n in enumerate(names):
            print(f"  {n:18s} {dur[:, k].mean():9.0f} cycles  {100 * dur[:, k].mean() / tot.mean():5.1f}%"
                  f"  (min {dur[:, k].min()}, max {dur[:, k].max()})")


if __name__ == "__main__":
    main()
