// Host entry points of attn_block.hip (device code: attn_block_dev.h).
#include "attn_block_dev.h"

using namespace ncf_attn;


#ifdef NCF_ATTN_STAMPS
// diagnostic builds only (not in ncf_hip.h): copy the phase stamps [2][1024][16] to the host
extern "C" int ncf_debug_attn_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_attn_stamps), sizeof(g_attn_stamps)) == hipSuccess
             ? NCF_OK
             : NCF_ERR_LAUNCH;
}
#endif

extern "C" int ncf_attn_block_supported(int64_t dim, int64_t heads, int64_t group_len) {
  if ((dim != 64 && dim != 128) || heads < 1 || dim % heads != 0) return 0;
  if (!hd_ok(dim, dim / heads)) return 0;
  return group_len >= 1 && group_len <= kMaxM ? 1 : 0;
}

extern "C" int ncf_attn_block_fwd(const float* xu, const float* xi, int64_t groups,
                                  int64_t group_len, int64_t heads, int64_t dim, const float* wq,
                                  const float* bq, const float* wk, const float* bk,
                                  const float* wv, const float* bv, const float* wo,
                                  const float* bo, float dropout_p, uint64_t seed,
                                  const ncf_step_clock* clock, float* q, float* k, float* v,
                                  float* probs, float* o, float* y, const int64_t* user_ids,
                                  void* stream) {
  NCF_CHECK_ARG(groups >= 0 && ncf_attn_block_supported(dim, heads, group_len),
                "ncf_attn_block_fwd: unsupported shape (D=%lld H=%lld M=%lld; need D=64 or 128, "
                "M<=%d)", (long long)dim, (long long)heads, (long long)group_len, kMaxM);
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_attn_block_fwd: dropout_p out of [0,1)");
  NCF_CHECK_ARG(y != nullptr && (q != nullptr) == (k != nullptr),
                "ncf_attn_block_fwd: q and k are given together (or neither)");
  NCF_CHECK_ARG(q == nullptr || probs != nullptr,
                "ncf_attn_block_fwd: a stashing forward needs probs (o may be NULL: the backward "
                "recomputes it from probs and v)");
  // the core runs unless the eval form applies (M == 1 without dropout: softmax == 1, o = v);
  // without q/k it stashes nothing (training with ncf_attn_block_bwd_rc)
  const int core = (q != nullptr || group_len > 1 || dropout_p > 0.0f) ? 1 : 0;
  const int share_q = kShareQ;
  const int64_t* uids = user_ids;   // (also the source rows of X_u: src_row)
  if (groups == 0) return NCF_OK;
  const int M = (int)group_len;
  const size_t lds = fwd_lds_d((int)dim, M);
  const dim3 grid((unsigned)ncf_cdiv(groups, groups_per_wg(dim)));
  hipStream_t st = (hipStream_t)stream;
  const float scale = sqrtf((float)(dim / heads));
#define NCF_ABF(D_, HD)                                                                          \
  if (dim == D_ && dim / heads == HD) {                                                          \
    static bool attr = false;                                                                    \
    if (!attr) { allow_lds(k_attn_block_fwd<D_, HD>, fwd_lds<D_>(kMaxM)); attr = true; }         \
    hipLaunchKernelGGL((k_attn_block_fwd<D_, HD>), grid, dim3(kThreads), lds, st, xu, xi, groups, \
                       M, wq, bq, wk, bk, wv, bv, wo, bo, scale, dropout_p, seed, clock, q, k, v, \
                       probs, o, y, core, uids, share_q);                                        \
  }
  NCF_ABF(64, 8)
  NCF_ABF(64, 16)
  NCF_ABF(64, 32)
  NCF_ABF(64, 64)
  NCF_ABF(128, 16)
  NCF_ABF(128, 32)
  NCF_ABF(128, 64)
#undef NCF_ABF
  NCF_CHECK_LAUNCH("ncf_attn_block_fwd");
  return NCF_OK;
}

// sized for either supported width (the larger of D = 64 / 128)
extern "C" int64_t ncf_attn_block_bwd_workspace(int64_t groups) {
  int64_t best = 0;
  for (int64_t D : {64, 128}) {
    const int64_t nb = groups <= 0 ? 1 : ncf_cdiv(groups, groups_per_wg(D));
    const int64_t PA = part_floats(D);
    const int64_t ws = nb * PA + ncf_reduce_scratch((int)nb, (int)PA) * 4;
    best = ws > best ? ws : best;
  }
  return best;
}

extern "C" int ncf_attn_block_bwd(const float* grad_y, const float* q, const float* k,
                                  const float* v, const float* probs, int64_t groups,
                                  int64_t group_len, int64_t heads, int64_t dim, const float* wq,
                                  const float* wk, const float* wv, const float* wo,
                                  float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                                  const float* o, const float* xu, const float* xi,
                                  float* const* grad_params, float* workspace,
                                  int64_t workspace_floats, ncf_reduce_list* defer,
                                  float* grad_q, float* grad_k, float* grad_v, float* grad_xu,
                                  float* grad_xi, const int64_t* user_ids, void* stream) {
  NCF_CHECK_ARG(groups >= 0 && ncf_attn_block_supported(dim, heads, group_len),
                "ncf_attn_block_bwd: unsupported shape (D=%lld H=%lld M=%lld; need D=64 or 128, "
                "M<=%d)", (long long)dim, (long long)heads, (long long)group_len, kMaxM);
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_attn_block_bwd: dropout_p out of [0,1)");
  const bool wg = grad_params != nullptr;
  NCF_CHECK_ARG(!wg || (xu && xi && workspace), "ncf_attn_block_bwd: the fused weight "
                "gradients need xu, xi and a workspace");
  NCF_CHECK_ARG(wg || (grad_q && grad_k && grad_v),
                "ncf_attn_block_bwd: without grad_params, grad_q/k/v are required");
  if (wg && workspace_floats < ncf_attn_block_bwd_workspace(groups)) {
    ncf_set_error("ncf_attn_block_bwd: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (groups == 0) return NCF_OK;
  const int M = (int)group_len, H = (int)heads;
  // (the forward recorded where it stashed Q once per group: the kernel reads that record)
  const int share_q = kShareQ;
  const size_t lds = bwd_lds_d((int)dim, M, H, wg);
  const int nb = (int)ncf_cdiv(groups, groups_per_wg(dim));
  const dim3 grid((unsigned)nb);
  hipStream_t st = (hipStream_t)stream;
  const float scale = sqrtf((float)(dim / heads));
  float* part = wg ? workspace : nullptr;
#define NCF_ABB(D_, HD)                                                                           \
  if (dim == D_ && dim / heads == HD) {                                                           \
    static bool attr = false;                                                                     \
    if (!attr) { allow_lds(k_attn_block_bwd<D_, HD, false>, bwd_lds<D_>(kMaxM, D_ / HD, true)); attr = true; } \
    hipLaunchKernelGGL((k_attn_block_bwd<D_, HD, false>), grid, dim3(kThreads), lds, st, grad_y, q, k, \
                       v, probs, groups, M, wq, wk, wv, wo, scale, dropout_p, seed, clock, o, xu, xi, \
                       part, grad_q, grad_k, grad_v, grad_xu, grad_xi, nullptr, nullptr, nullptr, user_ids, \
                       share_q);                                                                  \
  }
  NCF_ABB(64, 8)
  NCF_ABB(64, 16)
  NCF_ABB(64, 32)
  NCF_ABB(64, 64)
  NCF_ABB(128, 16)
  NCF_ABB(128, 32)
  NCF_ABB(128, 64)
#undef NCF_ABB
  NCF_CHECK_LAUNCH("ncf_attn_block_bwd");
  if (!wg) return NCF_OK;
  return defer_partials(dim, grad_params, part, nb, workspace, workspace_floats, defer, stream);
}

// the recompute backward holds the recomputed probabilities beside dS in LDS
extern "C" int ncf_attn_block_rc_supported(int64_t dim, int64_t heads, int64_t group_len) {
  return ncf_attn_block_supported(dim, heads, group_len) &&
                 bwd_lds_d((int)dim, (int)group_len, (int)heads, true, true) <= kMaxLds
             ? 1
             : 0;
}

extern "C" int ncf_attn_block_bwd_rc(const float* grad_y, const float* xu, const float* xi,
                                     int64_t groups, int64_t group_len, int64_t heads,
                                     int64_t dim, const float* wq, const float* bq,
                                     const float* wk, const float* bk, const float* wv,
                                     const float* bv, const float* wo, float dropout_p,
                                     uint64_t seed, const ncf_step_clock* clock,
                                     float* const* grad_params, float* workspace,
                                     int64_t workspace_floats, ncf_reduce_list* defer,
                                     float* grad_xu, float* grad_xi, const int64_t* user_ids,
                                     void* stream) {
  NCF_CHECK_ARG(groups >= 0 && ncf_attn_block_supported(dim, heads, group_len),
                "ncf_attn_block_bwd_rc: unsupported shape (D=%lld H=%lld M=%lld; need D=64 or "
                "128, M<=%d)", (long long)dim, (long long)heads, (long long)group_len, kMaxM);
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_attn_block_bwd_rc: dropout_p out of [0,1)");
  NCF_CHECK_ARG(grad_y && xu && xi && wq && bq && wk && bk && wv && bv && wo && grad_params &&
                    workspace && grad_xu && grad_xi,
                "ncf_attn_block_bwd_rc: null argument");
  if (workspace_floats < ncf_attn_block_bwd_workspace(groups)) {
    ncf_set_error("ncf_attn_block_bwd_rc: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  NCF_CHECK_ARG(ncf_attn_block_rc_supported(dim, heads, group_len),
                "ncf_attn_block_bwd_rc: M=%lld H=%lld needs more LDS than a workgroup has",
                (long long)group_len, (long long)heads);
  if (groups == 0) return NCF_OK;
  const int M = (int)group_len, H = (int)heads;
  const int share_q = kShareQ;
  const int64_t* uids = user_ids;
  const size_t lds = bwd_lds_d((int)dim, M, H, true, true);
  const int nb = (int)ncf_cdiv(groups, groups_per_wg(dim));
  const dim3 grid((unsigned)nb);
  hipStream_t st = (hipStream_t)stream;
  const float scale = sqrtf((float)(dim / heads));
#define NCF_ABR(D_, HD)                                                                           \
  if (dim == D_ && dim / heads == HD) {                                                           \
    static bool attr = false;                                                                     \
    if (!attr) { allow_lds(k_attn_block_bwd<D_, HD, true>, bwd_lds<D_>(kMaxM, D_ / HD, true, true) <= kMaxLds ? bwd_lds<D_>(kMaxM, D_ / HD, true, true) : kMaxLds); attr = true; } \
    hipLaunchKernelGGL((k_attn_block_bwd<D_, HD, true>), grid, dim3(kThreads), lds, st, grad_y,     \
                       nullptr, nullptr, nullptr, nullptr, groups, M, wq, wk, wv, wo, scale,       \
                       dropout_p, seed, clock, nullptr, xu, xi, workspace, nullptr, nullptr,       \
                       nullptr, grad_xu, grad_xi, bq, bk, bv, uids, share_q);                      \
  }
  NCF_ABR(64, 8)
  NCF_ABR(64, 16)
  NCF_ABR(64, 32)
  NCF_ABR(64, 64)
  NCF_ABR(128, 16)
  NCF_ABR(128, 32)
  NCF_ABR(128, 64)
#undef NCF_ABR
  NCF_CHECK_LAUNCH("ncf_attn_block_bwd_rc");
  return defer_partials(dim, grad_params, workspace, nb, workspace, workspace_floats, defer, stream);
}
