"""ctypes binding of libncf_hip.so (include/ncf_hip.h).

The library is built for gfx950 by ``build_ext.sh`` (driven by ``__graft_entry__.build()``) and
lives next to this file.  It links ``libamdhip64.so.7``; ``torch`` is imported first so the
dynamic linker binds the library to the SAME HIP runtime torch uses, which makes torch's stream
handles and device pointers valid inside it.

There is no CPU fallback: if the library is missing or cannot be loaded, every compute entry
point raises ``NCFLibraryError``.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL: binds libncf_hip to torch's HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "libncf_hip.so")
LIB_PATH = os.environ.get("NCF_HIP_LIB") or _DEFAULT_LIB   # env: A/B builds


class NCFLibraryError(RuntimeError):
    pass


P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
F32 = ctypes.c_float
F64 = ctypes.c_double
U64 = ctypes.c_uint64

# name -> (restype, argtypes); mirrors include/ncf_hip.h exactly
SIGNATURES = {
    "ncf_version": (I32, []),
    "ncf_last_error": (ctypes.c_char_p, []),
    "ncf_event_create": (I32, [P]),
    "ncf_event_create_scoped": (I32, [P, I32]),
    "ncf_event_destroy": (I32, [P]),
    "ncf_event_record": (I32, [P, P]),
    "ncf_stream_wait_event": (I32, [P, P]),
    "ncf_event_synchronize": (I32, [P]),
    "ncf_memcpy_async": (I32, [P, P, I64, P]),
    "ncf_device_count": (I32, []),
    "ncf_build_info": (ctypes.c_char_p, []),
    "ncf_gather_ln_gmf_ld_fwd": (I32, [P, P, I64, P, P, P, P, I64, I64, I64, I64, P, P, P, P, P, P,
                                       F32, I64, P, P, P, P, P, P, P]),
    "ncf_gather_ln_gmf_fwd": (I32, [P, P, I64, P, P, P, P, I64, I64, I64, P, P, P, P, P, P, F32,
                                    P, P, P, P, P, P, P]),
    "ncf_gather_ln_gmf_scaled_fwd": (I32, [P, P, I64, P, P, P, P, I64, I64, I64, P, P, P, P, P, P,
                                           F32, P, F32, I64, P, P, P, P, P, P, P]),
    "ncf_gather_ln_gmf_bf16_fwd": (I32, [P, P, I64, P, P, P, P, I64, I64, I64, P, P, P, P, P, P,
                                         F32, I64, P, P, P, P, P, P, P]),
    "ncf_gather_rows": (I32, [P, I64, P, I64, I64, P, P, F32, P, P, P]),
    "ncf_gemm_f32": (I32, [I64, I64, I64, P, I64, I32, P, I64, I32, P, I64, P, I32, P]),
    "ncf_gemm_splitk_workspace": (I64, [I64, I64, I32]),
    "ncf_gemm_f32_splitk": (I32, [I64, I64, I64, P, I64, I32, P, I64, I32, P, I64, I32, P, I32,
                                  P, I64, P, P]),
    "ncf_gemm_direct": (I32, [I64, I64, I64, P, I64, I32, P, I64, I32, P, I64, P, I32, P]),
    "ncf_gemm_rows": (I32, [I64, I64, I64, P, I64, P, I64, I32, P, I64, P, I32, P]),
    "ncf_wgrad_grouped_workspace": (I64, [P, I32]),
    "ncf_wgrad_grouped": (I32, [P, I32, P, I64, P, P]),
    "ncf_reduce_batch_scratch": (I64, [P]),
    "ncf_reduce_set_vec": (I64, [I64]),
    "ncf_stream_spin": (I32, [I64, P]),
    "ncf_stream_create_cu_mask": (I32, [I32, P]),
    "ncf_stream_destroy": (I32, [P]),
    "ncf_adam_sweep_set_blocks": (I64, [I64]),
    "ncf_dropout_rows": (I32, [P, I64, I64, I64, F32, U64, P, P, P]),
    "ncf_reduce_batch": (I32, [P, P, I64, P]),
    "ncf_colsum_workspace": (I64, [I64, I64]),
    "ncf_colsum": (I32, [P, I64, I64, I64, P, I32, P, I64, P]),
    "ncf_attention_fwd": (I32, [P, P, P, I64, I64, I64, I64, F32, U64, P, P, P, P]),
    "ncf_attention_fwd_masked": (I32, [P, P, P, I64, I64, I64, I64, F32, U64, P, P, P, P, P]),
    "ncf_attention_bwd": (I32, [P, P, P, P, P, I64, I64, I64, I64, F32, U64, P, P, P, P, P, P]),
    "ncf_attn_block_supported": (I32, [I64, I64, I64]),
    "ncf_mlp_fused_supported": (I32, [I64, I64, P]),
    "ncf_attn_mlp_fused_supported": (I32, [I64, I64, I64, I64, P]),
    "ncf_attn_mlp_fwd": (I32, [P, P, I64, I64, P, P, P, P, P, P, P, P, F32, U64, P, P, P, P, P, P,
                               P, P, I64, P, F32, P, P, P, P, P, P, P, I32, P]),
    "ncf_attn_mlp_bwd": (I32, [I64, I64, P, P, I64, P, F32, U64, P, P, P, I64, P, P, P, P, P, P,
                               P, P, P, P, P, P, I64, P, P, P, P, I32, P]),
    "ncf_attn_mlp_fwd_small": (I32, [P, P, I64, I64, P, P, P, P, P, P, P, P, F32, U64, P, P, P, P, P, P,
                               P, P, I64, P, F32, P, P, P, P, P, P, P, I32, P]),
    "ncf_attn_mlp_bwd_small": (I32, [I64, I64, P, P, I64, P, F32, U64, P, P, P, I64, P, P, P, P, P, P,
                               P, P, P, P, P, P, I64, P, P, P, P, I32, P]),
    "ncf_attn_mlp_bwd_workspace": (I64, [I64, I32]),
    "ncf_attn_mlp_bwd_workspace_small": (I64, [I64, I32]),
    "ncf_attn_mlp_fused_supported_small": (I32, [I64, I64, I64, I64, P]),
    "ncf_alias_build": (I32, [P, I64, P, P]),
    "ncf_group_metrics_workspace": (I64, [I64, I64]),
    "ncf_group_metrics": (I32, [P, P, I64, I64, P, I64, F32, P, P, I64, P]),
    "ncf_auc_count": (I32, [P, P, I64, P, I64, P, P]),
    "ncf_embedding_export": (I32, [P, I64, P, I64, I64, P, P, F32, I32, P, P, P]),
    "ncf_sample_negatives": (I32, [P, P, I64, I64, P, P, I64, P, P, I64, U64, I64, P, P, P, P, P]),
    "ncf_mlp_fwd": (I32, [P, I64, I64, P, I64, P, F32, F32, U64, P, P, P, P, P, P, P, P, P]),
    "ncf_mlp_fwd_bf16": (I32, [P, I64, I64, P, I64, P, F32, F32, U64, P, P, P, P, P, P, P, P, P]),
    "ncf_mlp_bwd_bf16": (I32, [P, I64, I64, P, P, I64, P, F32, U64, P, P, P, P, I64, P, P]),
    "ncf_mlp_fwd_split": (I32, [P, I64, I64, P, I64, P, F32, F32, U64, P, P, P, P, P, P, P, P, P]),
    "ncf_mlp_bwd_split": (I32, [P, I64, I64, P, P, I64, P, F32, U64, P, P, P, P, I64, P, P]),
    "ncf_mlp_bwd_workspace": (I64, [I64]),
    "ncf_mlp_bwd": (I32, [P, I64, I64, P, P, I64, P, F32, U64, P, P, P, P, I64, P, P]),
    "ncf_attn_block_fwd": (I32, [P, P, I64, I64, I64, I64, P, P, P, P, P, P, P, P, F32, U64, P,
                                 P, P, P, P, P, P, P, P]),
    "ncf_attn_block_bwd_workspace": (I64, [I64]),
    "ncf_attn_block_rc_supported": (I32, [I64, I64, I64]),
    "ncf_attn_block_bwd_rc": (I32, [P, P, P, I64, I64, I64, I64, P, P, P, P, P, P, P, F32, U64, P,
                                    P, P, I64, P, P, P, P, P]),
    "ncf_attn_block_bwd": (I32, [P, P, P, P, P, I64, I64, I64, I64, P, P, P, P, F32, U64, P, P,
                                 P, P, P, P, I64, P, P, P, P, P, P, P, P]),
    "ncf_relu_ln_dropout_fwd": (I32, [P, I64, I64, P, P, F32, F32, U64, P, P, P, P, P]),
    "ncf_relu_ln_dropout_bwd_workspace": (I64, [I64, I64]),
    "ncf_relu_ln_dropout_bwd": (I32, [P, P, P, P, P, I64, I64, F32, U64, P, P, P, P, P, P, I64,
                                      P, P]),
    "ncf_head_fwd": (I32, [P, I64, I64, P, P, P, P, P, P, P, P]),
    "ncf_head_bwd_workspace": (I64, [I64, I64, I64]),
    "ncf_head_bwd": (I32, [P, P, P, P, P, P, I64, I64, P, P, P, P, I64, P, P, P, P, P, P, P, P,
                           P, P, P, F64, P, I64, P, P]),
    "ncf_embedding_bwd_workspace": (I64, [I64, I64]),
    "ncf_embedding_bwd": (I32, [P, P, I64, I64, I64, I64, P, P, P, P, P, P, P, P, P, P, F32, P, P,
                                P, P, P, P, P, P, P, P, P, P, P, P, I64, P]),
    "ncf_dedup_ids": (I32, [P, P, I64, I64, I64, I64, P, P, P, P, P, P, I64, P]),
    "ncf_dedup_set_small_max": (I64, [I64]),
    "ncf_dedup_ids2": (I32, [P, I64, I64, P, I64, I64, I64, P, P, P, P, P, P, I64, P]),
    "ncf_dedup_inverse": (I32, [I64, I64, I64, I64, I64, P, P, P, I64, P]),
    "ncf_shard_plan": (I32, [P, P, I64, I32, I64, I64, I64, P, P, I64, P, P]),
    "ncf_shard_owner_prepare": (I32, [P, P, ctypes.c_int32, P, P, P, P, I64, I64, P, P, P, P, P,
                                      P, P]),
    "ncf_shard_owner_gather": (I32, [P, P, P, P, I64, P, P, I64, I64, P, P]),
    "ncf_shard_owner_gradsum": (I32, [P, P, P, P, I64, I32, I64, P, P, P, P, P]),
    "ncf_shard_rows": (I32, [P, P, P, P, I64, I64, P, P, P, P, I32, P]),
    "ncf_comm_available": (I32, []),
    "ncf_comm_unique_id": (I32, [P, I64]),
    "ncf_comm_init": (I32, [P, I64, I32, I32, P]),
    "ncf_comm_destroy": (I32, [P]),
    "ncf_comm_alltoallv": (I32, [P, P, P, P, P, I64, P]),
    "ncf_comm_allreduce_sum_f32": (I32, [P, P, I64, P]),
    "ncf_embedding_bwd_reduce_rows": (I32, [I64, I64, I64, I64, P, P, P, P, P, P, P, P, P, P, F32,
                                            P, P, P, P, P, P, P, P, I64, I64, P, P, P, P, P, I64,
                                            P, P]),
    "ncf_embedding_bwd_reduce_apply_clock": (I32, [I64, I64, I64, I64, P, P, P, P, P, P, F32, P, P,
                                                   P, P, P, P, P, P, P, P, P, I64, P, P, I32, P,
                                                   P, F64, F64, F64, F64, P]),
    "ncf_embedding_bwd_reduce": (I32, [I64, I64, I64, I64, P, P, P, P, P, P, P, P, P, P, F32, P, P,
                                       P, P, P, P, P, P, P, P, P, I64, P, P]),
    "ncf_embedding_bwd_reduce_bf16": (I32, [I64, I64, I64, I64, P, P, P, P, P, P, P, P, P, P, F32,
                                            P, P, P, P, P, P, P, P, P, P, P, I64, P, P]),
    "ncf_slot_reset": (I32, [P, P, I32, P, I64, P]),
    "ncf_scatter_compact_rows": (I32, [P, I64, P, P, I32, P, I64, P]),
    "ncf_adam_table": (I32, [P, P, P, I64, I64, P, P, F64, F64, F64, F64, F64, F64, P]),
    "ncf_adam_flat": (I32, [P, P, P, P, I64, F64, F64, F64, F64, F64, F64, P]),
    "ncf_adam_table_dense_grad": (I32, [P, P, P, P, I64, F64, F64, F64, F64, F64, F64, P]),
    "ncf_fill_2d": (I32, [P, I64, I64, I64, F32, P]),
    "ncf_adam_step_scalars": (I32, [F64, F64, F64, F64, I64, I64, P]),
    "ncf_adam_rows_catchup": (I32, [P, P, P, P, P, P, I64, P, P, I32, I64, P, I32, P, F64, F64, F64,
                                    F64, P]),
    "ncf_adam_rows_apply": (I32, [P, P, P, P, P, P, P, P, I64, P, P, I32, I64, P, I32, P, F64, F64,
                                  F64, F64, P]),
    "ncf_adam_sweep": (I32, [P, P, P, P, P, P, I64, I64, I64, P, I32, P, F64, F64, F64, F64, P]),
    "ncf_step_clock_advance": (I32, [P, U64, P]),
    "ncf_step_clock_set": (I32, [P, I32, U64, P]),
    "ncf_adam_rows_catchup_clock": (I32, [P, P, P, P, P, P, I64, P, P, I32, I64, P, I32, P, P, F64,
                                          F64, F64, F64, P]),
    "ncf_adam_rows_apply_clock": (I32, [P, P, P, P, P, P, P, P, I64, P, P, I32, I64, P, I32, P, P,
                                        F64, F64, F64, F64, P]),
    "ncf_adam_sweep_rolling": (I32, [P, P, P, P, P, P, I64, I64, I32, I64, P, I32, P, P, F64, F64,
                                     F64, F64, P]),
    "ncf_adam_pairs_catchup_clock": (I32, [P, I32, I64, P, I64, I32, P, P, F64, F64, F64, F64, P]),
    "ncf_adam_pairs_catchup_lock_clock": (I32, [P, I32, I64, P, I64, I32, I32, P, P, F64, F64, F64,
                                                F64, P]),
    "ncf_adam_pairs_catchup_claim_clock": (I32, [P, I32, I64, P, P, I64, I32, P, P, F64, F64, F64,
                                                 F64, P]),
    "ncf_adam_pairs_apply_gsum_clock": (I32, [P, I32, I64, P, I64, I32, P, P, P, I32, P, P, F64,
                                              F64, F64, F64, P]),
    "ncf_adam_pairs_apply_clock": (I32, [P, I32, I64, P, I64, I32, P, P, F64, F64, F64, F64, P]),
    "ncf_adam_pairs_sweep_rolling": (I32, [P, I32, I64, I32, I32, P, P, F64, F64, F64, F64, P]),
    "ncf_adam_pairs_sweep_rolling_part": (I32, [P, I32, I64, I32, I32, I32, I32, P, P, F64, F64, F64,
                                                F64, P]),
    "ncf_adam_table_bf16": (I32, [P, P, P, I64, I64, P, P, F64, F64, F64, F64, F64, F64, P]),
    "ncf_adam_sweep_bf16": (I32, [P, P, P, P, P, P, I64, I64, I64, P, I32, P, F64, F64, F64, F64, P]),
    "ncf_adam_flat_clock": (I32, [P, P, P, P, I64, P, I32, P, F64, F64, F64, F64, P]),
    "ncf_adam_flat_clock_close": (I32, [P, P, P, P, I64, P, I32, P, F64, F64, F64, F64, U64, P]),
    "ncf_score_queries": (I32, [P, I64, P, I64, I64, P, P, F32, P, P, P, P, P]),
    "ncf_score_item_bias": (I32, [P, I64, P, P, P, P, P]),
    "ncf_score_kth": (I32, [P, I64, I64, I32, P, I64, P, P]),
    "ncf_score_sample_split16": (I32, [P, I64, P, I64, I64, I64, P, I64, I64, P, P]),
    "ncf_score_kth16": (I32, [P, I64, I64, I32, P, P]),
    "ncf_score_collect": (I32, [P, P, I64, P, P, I64, I64, P, I64, P, P, P]),
    "ncf_score_split_items": (I32, [P, I64, I64, P, P]),
    "ncf_score_collect_split": (I32, [P, P, I64, P, P, I64, I64, P, I64, P, P, I32, I64, P]),
    "ncf_score_item_norm_max": (I32, [P, I64, I64, P, P]),
    "ncf_score_margin": (I32, [P, P, I64, I64, P, F32, P, P]),
    "ncf_score_select_rescored": (I32, [P, I64, P, P, I64, I32, P, P, P, I64, P, F32, P, P, P,
                                        P, P, P]),
    "ncf_score_select": (I32, [P, I64, P, P, I64, I32, P, P, P, P, P]),
    "ncf_score_merge": (I32, [P, P, I64, I64, I32, P, P, P]),
    "ncf_temporal_fwd": (I32, [P, P, P, P, I64, P, P, P, P, I64, I64, P, P, P]),
    "ncf_temporal_bwd": (I32, [P, P, P, I64, P, I64, P, P, P, P]),
}


class ReduceDesc(ctypes.Structure):
    """ncf_reduce_desc (include/ncf_hip.h)."""
    _fields_ = [("part", P), ("out", P), ("stride", I64), ("ldo", I64), ("L", ctypes.c_int32),
                ("cols", ctypes.c_int32), ("P", ctypes.c_int32), ("accumulate", ctypes.c_int32),
                ("scale", F32), ("reserved", ctypes.c_int32)]


REDUCE_LIST_MAX = 64


class WgradDesc(ctypes.Structure):
    """ncf_wgrad_desc (include/ncf_hip.h)."""
    _fields_ = [("dy", P), ("x", P), ("dw", P), ("dbias", P), ("ldy", I64), ("ldx", I64),
                ("ldw", I64), ("m_out", ctypes.c_int32), ("k_in", ctypes.c_int32),
                ("n", ctypes.c_int32), ("slabs", ctypes.c_int32), ("accumulate", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


WGRAD_GROUP_MAX = 8


class MlpLayer(ctypes.Structure):
    """ncf_mlp_layer (include/ncf_hip.h)."""
    _fields_ = [("w", P), ("ldw", I64), ("b", P), ("gamma", P), ("beta", P), ("r", P), ("a", P),
                ("mean", P), ("rstd", P), ("dlin", P), ("dbias", P), ("dgamma", P), ("dbeta", P),
                ("dw", P)]


class HeadArgs(ctypes.Structure):
    """ncf_head_args (include/ncf_hip.h)."""
    _fields_ = [(f, P) for f in ("prob", "grad_prob", "targets", "mf_pred", "mlp_pred",
                                 "mf_user_ln", "mf_item_ln", "mlp_out_w", "final_w", "mf_out_w",
                                 "grad_mf_user_ln", "grad_mf_item_ln", "grad_mlp_out_w",
                                 "grad_mlp_out_b", "grad_mf_out_w", "grad_mf_out_b",
                                 "grad_final_w", "grad_final_b", "loss")] + \
        [("loss_denominator", ctypes.c_double), ("user_ids", P), ("group_rows", I64)]


class TablePair(ctypes.Structure):
    """ncf_table_pair (include/ncf_hip.h)."""
    _fields_ = [("p0", P), ("m0", P), ("v0", P), ("p1", P), ("m1", P), ("v1", P), ("g0", P),
                ("g1", P), ("row_ids", P), ("stamp", P), ("rows", I64), ("param_dtype", I64)]


DTYPE_F32, DTYPE_BF16 = 0, 1


SHARD_MAX_WORLD = 64


class ShardPlanOut(ctypes.Structure):
    """ncf_shard_plan_out (include/ncf_hip.h)."""
    _fields_ = [(f, P) for f in ("keys0", "keys1", "uniq0", "uniq1", "num_unique", "inv0", "inv1",
                                 "counts", "send", "spos0", "spos1", "bounds", "spos64_0",
                                 "spos64_1", "rows0", "rows1")]


class ShardRecv(ctypes.Structure):
    """ncf_shard_recv (include/ncf_hip.h): per source s, kind-0 entries at [start[s],
    start[s] + n0[s]), kind-1 entries up to start[s + 1]."""
    _fields_ = [("world", ctypes.c_int32), ("start", ctypes.c_int32 * (SHARD_MAX_WORLD + 1)),
                ("n0", ctypes.c_int32 * SHARD_MAX_WORLD)]


class ReduceList(ctypes.Structure):
    """ncf_reduce_list: deferred gradient reductions collected during one backward."""
    _fields_ = [("count", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("d", ReduceDesc * REDUCE_LIST_MAX)]

    @property
    def address(self) -> int:
        return ctypes.addressof(self)


_lock = threading.Lock()
_lib = None
_load_error = None


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes library; raise NCFLibraryError when unavailable."""
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            _load_error = f"{path} not found — run __graft_entry__.build() (or ./build_ext.sh)"
            raise NCFLibraryError(_load_error)
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            _load_error = f"cannot load {path}: {e}"
            raise NCFLibraryError(_load_error) from e
        check_build(lib, path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _bind_fast(lib)
        _lib = lib
        return lib


def build_info(lib) -> dict:
    """{"abi": .., "src": ..} compiled into the library (ncf_build_info)."""
    try:
        fn = lib.ncf_build_info
    except AttributeError:
        return {}
    fn.restype, fn.argtypes = ctypes.c_char_p, []
    return dict(kv.split("=", 1) for kv in fn().decode().split())


def check_build(lib, path: str = LIB_PATH):
    """Refuse a library built against another C-ABI table than SIGNATURES, or from other kernel
    sources than the ones beside this package (a stale build: _abi.py).  The sources are not
    checked when they are absent, nor for a library named by NCF_HIP_LIB (an A/B build from
    another source tree)."""
    from . import _abi
    info = build_info(lib)
    want_abi = _abi.abi_hash(SIGNATURES)
    if info.get("abi") != want_abi:
        raise NCFLibraryError(f"{path} was built against another C-ABI table (abi "
                              f"{info.get('abi')} != {want_abi}): rebuild (./build_ext.sh)")
    want_src = _abi.src_hash() if os.path.abspath(path) == _DEFAULT_LIB else ""
    if want_src and info.get("src") != want_src:
        raise NCFLibraryError(f"{path} is stale: built from other kernel sources (src "
                              f"{info.get('src')} != {want_src}): rebuild (./build_ext.sh)")


# name -> CPython wrapper of the entry point (_ncffast, built beside the library by
# build_ext.sh from SIGNATURES): the same call without ctypes' per-argument conversion
FAST = {}


# The CPython fast-call binding (_ncffast) when it is built (False: ctypes alone, A/B of host time)
FASTCALL = True


def _bind_fast(lib):
    if not FASTCALL:
        return
    try:
        from . import _ncffast
    except ImportError:
        return      # ctypes alone (same results; ~7 us more host time per call)
    for i, name in enumerate(_ncffast.NAMES):
        if name not in SIGNATURES:
            continue
        _ncffast.bind(i, ctypes.cast(getattr(lib, name), ctypes.c_void_p).value)
        FAST[name] = getattr(_ncffast, name)
    global _fast_mod
    _fast_mod = _ncffast if hasattr(_ncffast, "tape_new") else None


def exported_symbols():
    return list(SIGNATURES)


def check(rc: int, name: str):
    if rc != 0:
        msg = _lib.ncf_last_error().decode(errors="replace") if _lib is not None else ""
        if rc == -1:
            raise ValueError(f"{name}: {msg}")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


# Optional live instrumentation (bench.py): when PROFILE is a list, every call appends
# (name, args, start_event, end_event) recorded on torch's current stream around the launch.
PROFILE = None


def _invoke(lib, name, args):
    f = FAST.get(name)
    if f is not None:
        try:
            return f(*args)
        except TypeError:
            pass       # an argument the fast path does not take (e.g. a ctypes object)
    if _recording:     # a call the tape cannot hold: the recording is unusable
        _fast_mod.tape_invalidate()
    return getattr(lib, name)(*args)


# stream plumbing, not kernels: never bracketed by the instrumentation
_NOT_TIMED = frozenset(("ncf_event_record", "ncf_stream_wait_event", "ncf_memcpy_async"))


def call(name: str, *args):
    lib = _lib if _lib is not None else load()
    if PROFILE is not None and name not in _NOT_TIMED:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        rc = _invoke(lib, name, args)
        b.record()
        PROFILE.append((name, args, a, b))
    else:
        rc = _invoke(lib, name, args)
    if rc != 0:
        check(rc, name)
    return rc


def call_tagged(name: str, tags, *args):
    """call(name, *args) whose scalar arguments listed in ``tags`` ({argument index: tape slot})
    are per-step values: a launch tape recording this call replays them with the values given
    for those slots (LaunchTape.replay bases, after the pointer ranges)."""
    if _recording:
        for a, slot in tags.items():
            _fast_mod.tape_tag(a, slot)
    return call(name, *args)


def query(name: str, *args) -> int:
    lib = _lib if _lib is not None else load()
    if _recording:     # sizes / capabilities: not launches, never part of a tape
        prev = _fast_mod.tape_hold(1)
        try:
            return int(_invoke(lib, name, args))
        finally:
            _fast_mod.tape_hold(prev)
    return int(_invoke(lib, name, args))


# ---- launch tapes (gen_fastcall.py): a recorded sequence of C-ABI calls replayed from C
_recording = False
_fast_mod = None


class LaunchTape:
    """The C-ABI calls one region of host code makes, recorded while it runs for real and
    replayed later in the same order from C (no Python per call).  ``record(ranges)``: pointer
    arguments inside one of the (base, size) ranges are re-based at replay onto the bases given
    to ``replay`` (in the same order), every other argument is replayed as recorded.  Only
    entry points reached through the fast-call binding are recorded; anything else reached
    while recording makes the tape invalid (``valid`` False after the region)."""

    def __init__(self):
        if _fast_mod is None:
            raise NCFLibraryError("launch tapes need the fast-call binding (_ncffast)")
        self._h = _fast_mod.tape_new()
        self.valid = False
        self.calls = 0

    def record(self, ranges=()):
        """Context manager: record the calls of its body (which run as usual)."""
        return _TapeRecording(self, ranges)

    def size(self):
        """(calls, patched pointer arguments, valid)"""
        return _fast_mod.tape_size(self._h)

    def replay(self, bases=()):
        rc = _fast_mod.tape_replay(self._h, tuple(bases))
        if rc != 0:
            i, code = rc
            check(code, f"launch tape call {i}")


class _TapeRecording:
    def __init__(self, tape, ranges):
        self.tape = tape
        self.ranges = tuple(int(x) for x in ranges)

    def __enter__(self):
        global _recording
        _fast_mod.tape_begin(self.tape._h, self.ranges)
        _recording = True
        return self.tape

    def __exit__(self, *exc):
        global _recording
        _recording = False
        n, valid = _fast_mod.tape_end()
        self.tape.calls = n
        self.tape.valid = bool(valid) and exc[0] is None
        return False


def tapes_available() -> bool:
    if _lib is None:
        load()
    return _fast_mod is not None


# release scope of the stream-to-stream events (RawEvent(stream_only=True): the fork / join
# points of a step, never waited on by the host): 0 system, 1 device, 2 no fence of their own
# (hipEventDisableSystemFence: visibility to the host and other devices is what it drops; the
# waiting streams are on this device).  Each record on the step's main queue stalls it: C2
# fused step 0.3089-0.3103 ms with 0, 0.3107-0.3136 with 1, 0.3038-0.3050 with 2 (r3av_*; the
# GPU suite green under 1 and 2)
STREAM_EVENT_SCOPE = 2


class RawEvent:
    """A hipEvent_t (no timing) whose record / wait go through the C-ABI
    (ncf_event_record / ncf_stream_wait_event), so a launch tape holds them in order with the
    kernels.  Created and destroyed outside any tape.  ``stream_only``: only other streams of
    this device wait on it (no host wait, no host read behind it), so its record needs no
    system-scope release (STREAM_EVENT_SCOPE)."""
    __slots__ = ("h", "host_ok")

    def __init__(self, stream_only: bool = False):
        lib = _lib if _lib is not None else load()
        out = ctypes.c_void_p()
        scope = STREAM_EVENT_SCOPE if stream_only else 0
        check(lib.ncf_event_create_scoped(ctypes.byref(out), scope), "ncf_event_create_scoped")
        self.h = out.value
        self.host_ok = scope == 0

    def record(self, stream: int):
        call("ncf_event_record", self.h, stream)

    def wait(self, stream: int):
        """``stream`` waits for the work recorded before the last record()."""
        call("ncf_stream_wait_event", stream, self.h)

    def synchronize(self):
        """Host wait (never part of a tape)."""
        if not self.host_ok:
            raise RuntimeError("RawEvent: a stream-only event has no host wait")
        check(_lib.ncf_event_synchronize(self.h), "ncf_event_synchronize")

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h and _lib is not None:
            try:
                _lib.ncf_event_destroy(h)
            except Exception:
                pass


def streams_overlap(side, main, us: int = 400) -> bool:
    """Whether work on torch stream `side` runs beside work on `main` (same device): a spin of
    `us` microseconds on each, timed on `main`; sharing a hardware queue serialises them (about
    two spans instead of one).  Host-synchronising; never call it under stream capture."""
    dt = 0.0
    for _ in range(2):        # (the first pass pays the kernel's first launch)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(main)
        side.wait_event(e0)
        call("ncf_stream_spin", us, side.cuda_stream)
        call("ncf_stream_spin", us, main.cuda_stream)
        main.wait_stream(side)
        e1.record(main)
        e1.synchronize()
        dt = e0.elapsed_time(e1) * 1e3
    return dt < 1.5 * us


# Side streams tried before giving up on one that runs beside the step's stream
SIDE_STREAM_TRIES = 8


_MASKED = []     # CU-masked streams made here (alive for the process)


def masked_stream(device, keep_per8: int):
    """A torch stream (ExternalStream) whose kernels use `keep_per8` of every 8 CUs."""
    out = ctypes.c_void_p()
    lib = _lib if _lib is not None else load()
    with torch.cuda.device(device):
        check(lib.ncf_stream_create_cu_mask(int(keep_per8), ctypes.byref(out)),
              "ncf_stream_create_cu_mask")
    s = torch.cuda.ExternalStream(out.value, device=device)
    _MASKED.append(s)
    return s


def side_stream(device, priority: int = 0, main=None):
    """A torch stream from the pool that runs beside `main` (default: the device's current
    stream), checked with streams_overlap: with GPU_MAX_HW_QUEUES = 4 (HIP's default) every
    stream shares one of four hardware queues per process, and a side stream that lands on the
    step's own queue serialises the work meant to overlap it (the C2 step: 0.37 instead of 0.27
    ms).  Tries the pool's next streams (SIDE_STREAM_TRIES) and warns if none runs beside it.
    Under stream capture (no host sync allowed) the first stream is returned unchecked."""
    main = main or torch.cuda.current_stream(device)
    s = torch.cuda.Stream(device, priority=priority)
    if torch.cuda.is_current_stream_capturing():
        return s
    for _ in range(SIDE_STREAM_TRIES - 1):
        if streams_overlap(s, main):
            return s
        s = torch.cuda.Stream(device, priority=priority)
    if not streams_overlap(s, main):
        import warnings
        warnings.warn("ncf_amd: no side stream found that runs beside the step's stream "
                      "(hardware queues shared); overlapped work will serialise")
    return s


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_ptr(device=None) -> int:
    """Raw hipStream_t of torch's current stream on `device` (int, torch.device or None)."""
    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = device.index if device.index is not None else torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)
