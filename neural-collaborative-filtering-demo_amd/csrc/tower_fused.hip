// The attention block and the MLP tower of AdvancedNCF fused into one launch per direction, for
// the C2 training geometry: D = 64, groups of M = 5 rows, so the attention workgroup's 16
// interaction groups are exactly the tower workgroup's 80 rows.
//
// Reference: MultiHeadAttention as AdvancedNCF.forward applies it (src/model/architecture.py:
// 18-57, 315-326), then self.mlp / mlp_output / final (:230-252, :337-354).  The two phases are
// the very device code of attn_block.hip and mlp_tower.hip (attn_block_dev.h, mlp_tower_dev.h:
// the same arithmetic, the same bits as the two launches); what the fusion removes is the launch
// boundary between them and the attention output's round trip through HBM before the tower
// reads it (it is still written once: the tower backward's layer-0 weight gradient reads it).
//
// LDS: the attention phase uses the first 72.7 KB (its three row buffers, scores, Q tile) —
// inside the tower's buffer Q (83.2 KB) — and writes its output rows straight into the tower's
// input buffer P; one barrier, then the tower phase (125.4 KB in all: one workgroup per CU).
//
// tower_fused_small.hip compiles this file again with 3 groups (15 rows, one MFMA row tile) per
// workgroup and its entry points suffixed _small: the small-batch tiles (the reference's default
// batch of 256 groups fills 86 CUs instead of 16).
#include "attn_block_dev.h"
#include "mlp_tower_dev.h"

#ifndef NCF_TF
#define NCF_TF(name) name
#endif

namespace {

namespace A = ncf_attn;
namespace T = ncf_mlp;

constexpr int kD = 64, kM = 5;
constexpr int kGW = A::AG<kD>::kGroups;                 // attention groups per workgroup
constexpr int kVR = kGW * kM;                           // = the tower's rows per workgroup
constexpr int kRp = 16 * ((kGW * kM + 15) / 16);       // the attention's padded rows
static_assert(kVR <= T::kRows && kRp == T::kRows, "the attention groups fill the tower tile");
static_assert(A::kThreads == T::kThreads, "one workgroup shape");
// the attention forward's LDS (three row buffers, scores, Q tile) inside the tower's buffer Q
// when it fits (80-row tiles); else in a region of its own behind the tower's (small tiles)
constexpr size_t kAttnFwdFloats = 3 * kRp * A::AG<kD>::kPitch + kGW * 8 * A::kMaxM +
                                  16 * A::AG<kD>::kPitch;
constexpr bool kAttnInQ = kAttnFwdFloats <= (size_t)T::kRows * T::kPQ;
constexpr size_t kAttnFwdOff = kAttnInQ ? 0 : T::kLdsFwd / sizeof(float);

template <int HD, int MM>
__global__ __launch_bounds__(T::kThreads) void k_attn_mlp_fwd(
    const float* __restrict__ xu, const float* __restrict__ xi, int64_t B,
    const float* __restrict__ wq, const float* __restrict__ bq, const float* __restrict__ wk,
    const float* __restrict__ bk, const float* __restrict__ wv, const float* __restrict__ bv,
    const float* __restrict__ wo, const float* __restrict__ bo, float scale, float p_drop,
    uint64_t seed, const ncf_step_clock* clock, float* __restrict__ Q, float* __restrict__ K,
    float* __restrict__ V, float* __restrict__ P, float* __restrict__ Y,
    const int64_t* __restrict__ uids, T::TowerArgs a, float eps,
    const float* __restrict__ w_out, const float* __restrict__ b_out,
    const float* __restrict__ mf_pred, const float* __restrict__ w_fin,
    const float* __restrict__ b_fin, float* __restrict__ mlp_pred, float* __restrict__ prob) {
  extern __shared__ float lds[];
  float* x_tile = lds + T::kRows * T::kPQ;     // the tower's buffer P
  A::attn_block_fwd_body<kD, HD>(lds + kAttnFwdOff, xu, xi, B, kM, wq, bq, wk, bk, wv, bv, wo, bo,
                                 scale, p_drop, seed, clock, Q, K, V, P, nullptr, Y, 1, uids,
                                 A::kShareQ, x_tile, T::kPP);
  __syncthreads();
  T::mlp_fwd_body<kD, T::kRT, kVR, MM>(lds, Y, B * kM, a, eps, p_drop, clock, w_out, b_out,
                                       mf_pred, w_fin, b_fin, mlp_pred, prob, true);
}

// The backward, tower first: head + LayerNorm/ReLU/dropout + every weight gradient of the tower
// (mlp_bwd_body with dx = NULL: its input gradient stays in buffer P), one barrier, then the
// attention backward reading that dY tile from LDS (attn_block_bwd_body's dYl form; the tower
// gradient never goes through HBM).  Q/K/V/P from the forward's stash, O recomputed.
template <int HD, int MM>
__global__ __launch_bounds__(T::kThreads) void k_attn_mlp_bwd(
    int64_t B, T::TowerArgs a, float p_drop, const ncf_step_clock* clock,
    float* __restrict__ part_tower, ncf_head_args h, float inv_n, const float* __restrict__ Y,
    const float* __restrict__ Qg, const float* __restrict__ Kg, const float* __restrict__ Vg,
    const float* __restrict__ Pg, const float* __restrict__ wq, const float* __restrict__ wk,
    const float* __restrict__ wv, const float* __restrict__ wo, float scale, uint64_t seed,
    const float* __restrict__ xu, const float* __restrict__ xi, float* __restrict__ part_attn,
    float* __restrict__ dxu, float* __restrict__ dxi, const int64_t* __restrict__ uids) {
  extern __shared__ float lds[];
  T::mlp_bwd_body<kD, MM, kVR>(lds, nullptr, B * kM, a, p_drop, clock, nullptr, part_tower, h, 1,
                               inv_n, Y, 1);
  __syncthreads();
  A::attn_block_bwd_body<kD, HD, false, false>(lds, nullptr, Qg, Kg, Vg, Pg, B, kM, wq, wk, wv, wo, scale,
                                        p_drop, seed, clock, nullptr, xu, xi, part_attn, nullptr,
                                        nullptr, nullptr, dxu, dxi, nullptr, nullptr, nullptr, uids,
                                        A::kShareQ, lds + T::kRows * T::kPQ, T::kPP);
}

constexpr size_t kLdsFused = T::kLdsFwd + (kAttnInQ ? 0 : sizeof(float) * kAttnFwdFloats);
constexpr size_t kLdsFusedBwd = T::kLds;
static_assert(sizeof(float) * (5 * kRp * A::AG<kD>::kPitch + kGW * 8 * kM * kM) <= kLdsFusedBwd,
              "the attention backward (8 heads at most) fits the tower backward's LDS");
static_assert(kRp * A::AG<kD>::kPitch <= T::kRows * T::kPQ,
              "the attention backward's dY copy (S0) lies below the tower's dX tile");

// partial floats of the tower (which = 0; sized for either tower width, as
// ncf_mlp_bwd_workspace) and of the attention block (which = 1) for `groups` groups in this
// file's tiles
int64_t tf_workspace(int64_t groups, int which) {
  const int64_t nb = groups <= 0 ? 1 : ncf_cdiv(groups, kGW);
  if (which == 0) {
    constexpr int W = T::Lay<128>::kPartW;
    return nb * W + 2 * ncf_reduce_scratch((int)nb, W);
  }
  constexpr int64_t PA = A::AG<kD>::kPartAttn;
  return nb * PA + ncf_reduce_scratch((int)nb, (int)PA) * 4;
}

}  // namespace

extern "C" int64_t NCF_TF(ncf_attn_mlp_bwd_workspace)(int64_t groups, int32_t which) {
  return tf_workspace(groups, which);
}

extern "C" int NCF_TF(ncf_attn_mlp_fused_supported)(int64_t dim, int64_t heads, int64_t group_len,
                                                    int64_t n_layers, const int64_t* hidden) {
  // (head width <= 16: wider heads' attention registers on top of the tower's spill)
  return dim == kD && group_len == kM && heads >= 1 && dim % heads == 0 && dim / heads <= 16 &&
                 A::hd_ok(dim, dim / heads) && T::tower_ok(dim, n_layers, hidden)
             ? 1
             : 0;
}

// ncf_attn_block_fwd (training: Q/K/V/P stashed, O recomputed by the backward) followed by
// ncf_mlp_fwd on its output, in one launch; tower_mode 0 = fp32 MFMA (ncf_mlp_fwd), 1 = bf16
// (ncf_mlp_fwd_bf16), 3 = split operands (ncf_mlp_fwd_split).
extern "C" int NCF_TF(ncf_attn_mlp_fwd)(const float* xu, const float* xi, int64_t groups, int64_t heads,
                                const float* wq, const float* bq, const float* wk, const float* bk,
                                const float* wv, const float* bv, const float* wo, const float* bo,
                                float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                                float* q, float* k, float* v, float* probs, float* y,
                                const int64_t* user_ids, const ncf_mlp_layer* layers,
                                int64_t n_layers, const int64_t* hidden, float eps,
                                const float* mlp_out_w, const float* mlp_out_b,
                                const float* mf_pred, const float* final_w, const float* final_b,
                                float* mlp_pred, float* prob, int32_t tower_mode, void* stream) {
  NCF_CHECK_ARG(groups >= 0 && NCF_TF(ncf_attn_mlp_fused_supported)(kD, heads, kM, n_layers, hidden),
                "ncf_attn_mlp_fwd: unsupported shape (need D = 64, M = 5, hidden [256,128,64])");
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_attn_mlp_fwd: dropout_p out of [0,1)");
  NCF_CHECK_ARG(q && k && v && probs && y, "ncf_attn_mlp_fwd: the training stash (q, k, v, probs) "
                "and y are required");
  NCF_CHECK_ARG(tower_mode == 0 || tower_mode == 1 || tower_mode == 3,
                "ncf_attn_mlp_fwd: tower_mode 0, 1 or 3");
  if (groups == 0) return NCF_OK;
  T::TowerArgs a;
  const int rc = T::make_args(layers, seed, kD, a);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const float scale = sqrtf((float)(kD / heads));
  const dim3 grid((unsigned)ncf_cdiv(groups, kGW));
#define NCF_FUSED_FWD(HD_, MM_)                                                                   \
  if (kD / heads == HD_ && tower_mode == MM_) {                                                   \
    static bool attr = false;                                                                     \
    if (!attr) {                                                                                  \
      (void)hipFuncSetAttribute((const void*)k_attn_mlp_fwd<HD_, MM_>,                            \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsFused);      \
      attr = true;                                                                                \
    }                                                                                             \
    hipLaunchKernelGGL((k_attn_mlp_fwd<HD_, MM_>), grid, dim3(T::kThreads), kLdsFused, st, xu, xi,  \
                       groups, wq, bq, wk, bk, wv, bv, wo, bo, scale, dropout_p, seed, clock, q, k, \
                       v, probs, y, user_ids, a, eps, mlp_out_w, mlp_out_b, mf_pred, final_w,     \
                       final_b, mlp_pred, prob);                                                  \
  }
  NCF_FUSED_FWD(8, 0) NCF_FUSED_FWD(16, 0)
  NCF_FUSED_FWD(8, 1) NCF_FUSED_FWD(16, 1)
  NCF_FUSED_FWD(8, 3) NCF_FUSED_FWD(16, 3)
#undef NCF_FUSED_FWD
  NCF_CHECK_LAUNCH("ncf_attn_mlp_fwd");
  return NCF_OK;
}

// ncf_mlp_bwd (head fused, fused weight gradients, input gradient kept in LDS) followed by
// ncf_attn_block_bwd on that gradient, in one launch.  Arguments as those two calls take them
// (the tower's x is the attention output y); both partial sets are deferred into `defer`
// (required: the caller's ncf_reduce_batch runs them with the step's other reductions).
extern "C" int NCF_TF(ncf_attn_mlp_bwd)(int64_t groups, int64_t heads, const float* y,
                                const ncf_mlp_layer* layers, int64_t n_layers,
                                const int64_t* hidden, float dropout_p, uint64_t seed,
                                const ncf_step_clock* clock, const ncf_head_args* head,
                                float* tower_workspace, int64_t tower_workspace_floats,
                                const float* q, const float* k, const float* v, const float* probs,
                                const float* wq, const float* wk, const float* wv, const float* wo,
                                const float* xu, const float* xi, float* const* attn_grad_params,
                                float* attn_workspace, int64_t attn_workspace_floats,
                                float* grad_xu, float* grad_xi, const int64_t* user_ids,
                                ncf_reduce_list* defer, int32_t tower_mode, void* stream) {
  NCF_CHECK_ARG(groups >= 0 && NCF_TF(ncf_attn_mlp_fused_supported)(kD, heads, kM, n_layers, hidden),
                "ncf_attn_mlp_bwd: unsupported shape (need D = 64, M = 5, hidden [256,128,64])");
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_attn_mlp_bwd: dropout_p out of [0,1)");
  NCF_CHECK_ARG(tower_mode == 0 || tower_mode == 1 || tower_mode == 3,
                "ncf_attn_mlp_bwd: tower_mode 0, 1 or 3");
  NCF_CHECK_ARG(y && q && k && v && probs && wq && wk && wv && wo && xu && xi && attn_grad_params &&
                    grad_xu && grad_xi && head && defer,
                "ncf_attn_mlp_bwd: y, the stash, the weights, xu/xi, grad params, grad_xu/xi, the "
                "head arguments and a defer list are required");
  const int64_t n = groups * kM;
  if (tower_workspace_floats < tf_workspace(groups, 0) ||
      attn_workspace_floats < tf_workspace(groups, 1)) {
    ncf_set_error("ncf_attn_mlp_bwd: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (groups == 0) return NCF_OK;
  T::TowerArgs a;
  int rc = T::make_args(layers, seed, kD, a);
  if (rc) return rc;
  for (int l = 0; l < 3; ++l)
    if (!a.l[l].r || !a.l[l].mean || !a.l[l].rstd || !a.l[l].dgamma || !a.l[l].dbeta ||
        !a.l[l].dbias || !a.l[l].dw) {
      ncf_set_error("ncf_attn_mlp_bwd: layer %d needs r/mean/rstd/dbias/dgamma/dbeta/dw", l);
      return NCF_ERR_ARG;
    }
  const ncf_head_args h = *head;
  NCF_CHECK_ARG((h.grad_prob != nullptr) != (h.targets != nullptr),
                "ncf_attn_mlp_bwd: head needs exactly one of grad_prob / targets");
  NCF_CHECK_ARG(h.prob && h.mf_pred && h.mlp_pred && h.mf_user_ln && h.mf_item_ln &&
                    h.mlp_out_w && h.final_w && h.mf_out_w && h.grad_mf_user_ln &&
                    h.grad_mf_item_ln && h.grad_mlp_out_w && h.grad_mlp_out_b &&
                    h.grad_mf_out_w && h.grad_mf_out_b && h.grad_final_w && h.grad_final_b,
                "ncf_attn_mlp_bwd: incomplete head arguments");
  const double den = h.loss_denominator > 0 ? h.loss_denominator : (double)n;
  const float inv_n = den > 0 ? (float)(1.0 / den) : 0.0f;
  hipStream_t st = (hipStream_t)stream;
  const float scale = sqrtf((float)(kD / heads));
  const int nb = (int)ncf_cdiv(groups, kGW);
#define NCF_FUSED_BWD(HD_, MM_)                                                                   \
  if (kD / heads == HD_ && tower_mode == MM_) {                                                   \
    static bool attr = false;                                                                     \
    if (!attr) {                                                                                  \
      (void)hipFuncSetAttribute((const void*)k_attn_mlp_bwd<HD_, MM_>,                            \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsFusedBwd);   \
      attr = true;                                                                                \
    }                                                                                             \
    hipLaunchKernelGGL((k_attn_mlp_bwd<HD_, MM_>), dim3((unsigned)nb), dim3(T::kThreads),         \
                       kLdsFusedBwd, st, groups, a, dropout_p, clock, tower_workspace, h, inv_n,  \
                       y, q, k, v, probs, wq, wk, wv, wo, scale, seed, xu, xi, attn_workspace,     \
                       grad_xu, grad_xi, user_ids);                                               \
  }
  NCF_FUSED_BWD(8, 0) NCF_FUSED_BWD(16, 0)
  NCF_FUSED_BWD(8, 1) NCF_FUSED_BWD(16, 1)
  NCF_FUSED_BWD(8, 3) NCF_FUSED_BWD(16, 3)
#undef NCF_FUSED_BWD
  NCF_CHECK_LAUNCH("ncf_attn_mlp_bwd");
  rc = T::defer_tower<kD>(a, head, h, inv_n, true, nb, tower_workspace, defer);
  if (rc) return rc;
  return A::defer_partials(kD, attn_grad_params, attn_workspace, nb, attn_workspace,
                           attn_workspace_floats, defer, stream);
}
