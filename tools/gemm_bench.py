"""Micro-benchmark of the fp32 MFMA GEMM variants on the C2 train-step shapes (GPU only).

    python tools/gemm_bench.py
Prints one line per (shape, variant): average device time over 50 launches (torch events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402

_ncf_pkg.load()
from ncf_amd import _lib  # noqa: E402

DEV = torch.device("cuda")
N_ROWS = 20480
# (name, M, N, K, a_trans, b_trans): forward Y = X·Wᵀ, dX = dY·W, dW = dYᵀ·X
SHAPES = [
    ("att_fwd 64x64", N_ROWS, 64, 64, 0, 1),
    ("mlp1_fwd 64->256", N_ROWS, 256, 64, 0, 1),
    ("mlp2_fwd 256->128", N_ROWS, 128, 256, 0, 1),
    ("mlp3_fwd 128->64", N_ROWS, 64, 128, 0, 1),
    ("mlp3_dX", N_ROWS, 128, 64, 0, 0),
    ("mlp2_dX", N_ROWS, 256, 128, 0, 0),
    ("mlp1_dX", N_ROWS, 64, 256, 0, 0),
    ("att_dX", N_ROWS, 64, 64, 0, 0),
    ("infer mlp1 65536", 65536, 256, 64, 0, 1),
]
WGRAD = [("mlp3_dW", 64, 128), ("mlp2_dW", 128, 256), ("mlp1_dW", 256, 64), ("att_dW", 64, 64)]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    st = _lib.stream_ptr(DEV)
    for name, M, N, K, at, bt in SHAPES:
        A = torch.randn(K, M, device=DEV) if at else torch.randn(M, K, device=DEV)
        B = torch.randn(N, K, device=DEV) if bt else torch.randn(K, N, device=DEV)
        C = torch.empty(M, N, device=DEV)
        lda, ldb = (M if at else K), (K if bt else N)
        flops = 2.0 * M * N * K
        ref = None
        for fn_name in ("ncf_gemm_f32", "ncf_gemm_direct", "ncf_gemm_rows"):
            if fn_name == "ncf_gemm_rows":
                if at:
                    continue
                fn = lambda: _lib.call(fn_name, M, N, K, A.data_ptr(), lda, B.data_ptr(), ldb, bt,  # noqa: E731
                                       C.data_ptr(), N, None, 0, st)
            else:
                fn = lambda: _lib.call(fn_name, M, N, K, A.data_ptr(), lda, at, B.data_ptr(), ldb,  # noqa: E731
                                       bt, C.data_ptr(), N, None, 0, st)
            C.zero_()
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = C.clone()
            err = (C - ref).abs().max().item()
            us = timeit(fn)
            print(f"{name:20s} {fn_name:22s} {us:8.2f} us  {flops / us / 1e6:7.1f} TF/s  maxdiff {err:.2e}",
                  flush=True)
    for name, Mo, Ko in WGRAD:
        dY = torch.randn(N_ROWS, Mo, device=DEV)
        X = torch.randn(N_ROWS, Ko, device=DEV)
        C = torch.empty(Mo, Ko, device=DEV)
        db = torch.empty(Mo, device=DEV)
        flops = 2.0 * Mo * Ko * N_ROWS
        for splits in (16, 40, 80, 160, 320):
            ws = torch.empty(max(_lib.query("ncf_gemm_splitk_workspace", Mo, Ko, splits),
                                 0), device=DEV)
            us1 = timeit(lambda: _lib.call("ncf_gemm_f32_splitk", Mo, Ko, N_ROWS, dY.data_ptr(), Mo, 1,
                                           X.data_ptr(), Ko, 0, C.data_ptr(), Ko, 0, None, splits,
                                           ws.data_ptr(), ws.numel(), None, st))
            print(f"{name:20s} splits={splits:4d} tiled {us1:8.2f} us ({flops / us1 / 1e6:6.1f} TF/s)",
                  flush=True)


if __name__ == "__main__":
    main()
