// Multi-head attention core over the M samples of one interaction group.
//
// Reference: MultiHeadAttention.forward, src/model/architecture.py:35-57, as used by
// AdvancedNCF.forward :315-326 (q = LN(user_mlp rows), k = v = LN(item_mlp rows), groups of
// M = 1 + negative_samples rows, mask=None).  scores = (q·kᵀ)/sqrt(hd) (:33, :45),
// softmax (:50), dropout on the weights (:51, nn.Dropout: keep-scale 1/(1-p)), ·v (:54),
// heads merged (:55).  The Q/K/V/out projections are MFMA GEMMs (gemm.hip); this file is the
// per-group core, which at M = 5 is far too small for MFMA: one lane owns one (group, head,
// query) row and keeps its scores in registers.
//
// Layout: Q, K, V, O are [N, D] row-major with N = B*L; head h owns columns [h*hd, (h+1)*hd).
// P (saved for backward) is the pre-dropout softmax [B, H, L, L].
//
// Mask (ncf_attention_fwd_masked; :47-48 scores.masked_fill(mask == 0, -inf)): a [B, H, L, L]
// byte per score, 0 = masked.  A masked score is -inf before the softmax, so its probability is
// exactly 0 and the backward needs no mask (dS = P (dP - sum P dP) is 0 there); a row with every
// score masked is NaN, as torch's softmax over all -inf makes it.
#include "ncf_common.h"

namespace {

template <int HD, int LMAX>
__global__ __launch_bounds__(256) void k_attn_fwd(const float* __restrict__ Q,
                                                  const float* __restrict__ Kt,
                                                  const float* __restrict__ V, int64_t B, int L,
                                                  int H, float scale, float p_drop,
                                                  uint64_t seed, const ncf_step_clock* clock, float* __restrict__ P,
                                                  float* __restrict__ O,
                                                  const uint8_t* __restrict__ mask) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * H * L) return;
  if (clock) seed += clock->seed;  // per-step stream of a captured step
  const int i = (int)(t % L);
  const int h = (int)((t / L) % H);
  const int64_t b = t / ((int64_t)L * H);
  const int D = H * HD;
  const float* q = Q + (b * L + i) * D + h * HD;
  float qr[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) qr[d] = q[d];
  float s[LMAX];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    if (j < L) {
      const float* k = Kt + (b * L + j) * D + h * HD;
      float acc = 0.0f;
#pragma unroll
      for (int d = 0; d < HD; ++d) acc = fmaf(qr[d], k[d], acc);
      s[j] = acc / scale;
      if (mask && mask[t * L + j] == 0) s[j] = -INFINITY;
      mx = fmaxf(mx, s[j]);
    }
  }
  float sum = 0.0f;
#pragma unroll
  for (int j = 0; j < LMAX; ++j)
    if (j < L) {
      s[j] = mx == -INFINITY ? NAN : expf(s[j] - mx);
      sum += s[j];
    }
  float o[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) o[d] = 0.0f;
  const float inv_keep = p_drop > 0.0f ? 1.0f / (1.0f - p_drop) : 1.0f;
  float* prow = P + t * L;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    if (j < L) {
      const float pj = s[j] / sum;
      prow[j] = pj;
      const float pd = p_drop > 0.0f ? pj * ncf_dropout_scale(seed, (uint64_t)t * L + j, p_drop, inv_keep) : pj;
      const float* v = V + (b * L + j) * D + h * HD;
#pragma unroll
      for (int d = 0; d < HD; ++d) o[d] = fmaf(pd, v[d], o[d]);
    }
  }
  float* orow = O + (b * L + i) * D + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) orow[d] = o[d];
}

// dS and dQ: one lane per (group, head, query row)
template <int HD, int LMAX>
__global__ __launch_bounds__(256) void k_attn_bwd_q(const float* __restrict__ dO,
                                                    const float* __restrict__ Kt,
                                                    const float* __restrict__ V,
                                                    const float* __restrict__ P, int64_t B, int L,
                                                    int H, float scale, float p_drop, uint64_t seed, const ncf_step_clock* clock,
                                                    float* __restrict__ dS, float* __restrict__ dQ) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * H * L) return;
  if (clock) seed += clock->seed;  // per-step stream of a captured step
  const int i = (int)(t % L);
  const int h = (int)((t / L) % H);
  const int64_t b = t / ((int64_t)L * H);
  const int D = H * HD;
  float g[HD];
  const float* go = dO + (b * L + i) * D + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) g[d] = go[d];
  const float inv_keep = p_drop > 0.0f ? 1.0f / (1.0f - p_drop) : 1.0f;
  const float* prow = P + t * L;
  float dp[LMAX];
  float tsum = 0.0f;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    if (j < L) {
      const float* v = V + (b * L + j) * D + h * HD;
      float acc = 0.0f;
#pragma unroll
      for (int d = 0; d < HD; ++d) acc = fmaf(g[d], v[d], acc);
      if (p_drop > 0.0f) acc *= ncf_dropout_scale(seed, (uint64_t)t * L + j, p_drop, inv_keep);
      dp[j] = acc;
      tsum = fmaf(prow[j], acc, tsum);
    }
  }
  float dq[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) dq[d] = 0.0f;
  float* dsrow = dS + t * L;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    if (j < L) {
      const float ds = prow[j] * (dp[j] - tsum);
      dsrow[j] = ds;
      const float* k = Kt + (b * L + j) * D + h * HD;
#pragma unroll
      for (int d = 0; d < HD; ++d) dq[d] = fmaf(ds, k[d], dq[d]);
    }
  }
  float* out = dQ + (b * L + i) * D + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) out[d] = dq[d] / scale;
}

// dK and dV: one lane per (group, head, key row)
template <int HD>
__global__ __launch_bounds__(256) void k_attn_bwd_kv(const float* __restrict__ Q,
                                                     const float* __restrict__ dO,
                                                     const float* __restrict__ P,
                                                     const float* __restrict__ dS, int64_t B,
                                                     int L, int H, float scale, float p_drop,
                                                     uint64_t seed, const ncf_step_clock* clock, float* __restrict__ dK,
                                                     float* __restrict__ dV) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * H * L) return;
  if (clock) seed += clock->seed;  // per-step stream of a captured step
  const int j = (int)(t % L);
  const int h = (int)((t / L) % H);
  const int64_t b = t / ((int64_t)L * H);
  const int D = H * HD;
  const float inv_keep = p_drop > 0.0f ? 1.0f / (1.0f - p_drop) : 1.0f;
  float dk[HD], dv[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) { dk[d] = 0.0f; dv[d] = 0.0f; }
  const int64_t bh = b * H + h;
  for (int i = 0; i < L; ++i) {
    const int64_t row = (bh * L + i);
    const float ds = dS[row * L + j];
    float pd = P[row * L + j];
    if (p_drop > 0.0f) pd *= ncf_dropout_scale(seed, (uint64_t)row * L + j, p_drop, inv_keep);
    const float* q = Q + (b * L + i) * D + h * HD;
    const float* go = dO + (b * L + i) * D + h * HD;
#pragma unroll
    for (int d = 0; d < HD; ++d) {
      dk[d] = fmaf(ds, q[d], dk[d]);
      dv[d] = fmaf(pd, go[d], dv[d]);
    }
  }
  float* ok = dK + (b * L + j) * D + h * HD;
  float* ov = dV + (b * L + j) * D + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    ok[d] = dk[d] / scale;
    ov[d] = dv[d];
  }
}

template <int HD, int LMAX>
int fwd_l(const float* Q, const float* K, const float* V, int64_t B, int L, int H, float p,
          uint64_t seed, const ncf_step_clock* clock, float* P, float* O, hipStream_t st,
          const uint8_t* mask) {
  const int64_t n = B * H * L;
  hipLaunchKernelGGL((k_attn_fwd<HD, LMAX>), dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, Q, K, V, B,
                     L, H, sqrtf((float)HD), p, seed, clock, P, O, mask);
  NCF_CHECK_LAUNCH("ncf_attention_fwd");
  return NCF_OK;
}

template <int HD, int LMAX>
int bwd_l(const float* Q, const float* K, const float* V, const float* P, const float* dO,
          int64_t B, int L, int H, float p, uint64_t seed, const ncf_step_clock* clock, float* dS, float* dQ, float* dK,
          float* dV, hipStream_t st) {
  const int64_t n = B * H * L;
  const float scale = sqrtf((float)HD);
  hipLaunchKernelGGL((k_attn_bwd_q<HD, LMAX>), dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, dO, K, V,
                     P, B, L, H, scale, p, seed, clock, dS, dQ);
  NCF_CHECK_LAUNCH("ncf_attention_bwd(q)");
  hipLaunchKernelGGL((k_attn_bwd_kv<HD>), dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, Q, dO, P, dS,
                     B, L, H, scale, p, seed, clock, dK, dV);
  NCF_CHECK_LAUNCH("ncf_attention_bwd(kv)");
  return NCF_OK;
}

template <int HD>
int fwd_hd(const float* Q, const float* K, const float* V, int64_t B, int L, int H, float p,
           uint64_t seed, const ncf_step_clock* clock, float* P, float* O, hipStream_t st,
           const uint8_t* mask) {
  if (L <= 8) return fwd_l<HD, 8>(Q, K, V, B, L, H, p, seed, clock, P, O, st, mask);
  return fwd_l<HD, 64>(Q, K, V, B, L, H, p, seed, clock, P, O, st, mask);
}

template <int HD>
int bwd_hd(const float* Q, const float* K, const float* V, const float* P, const float* dO,
           int64_t B, int L, int H, float p, uint64_t seed, const ncf_step_clock* clock, float* dS, float* dQ, float* dK,
           float* dV, hipStream_t st) {
  if (L <= 8) return bwd_l<HD, 8>(Q, K, V, P, dO, B, L, H, p, seed, clock, dS, dQ, dK, dV, st);
  return bwd_l<HD, 64>(Q, K, V, P, dO, B, L, H, p, seed, clock, dS, dQ, dK, dV, st);
}

}  // namespace

static int attention_fwd(const float* q, const float* k, const float* v, int64_t groups,
                         int64_t group_len, int64_t heads, int64_t dim, float dropout_p,
                         uint64_t seed, const ncf_step_clock* clock, float* probs, float* out,
                         const uint8_t* mask, void* stream) {
  NCF_CHECK_ARG(groups >= 0 && group_len >= 1 && group_len <= 64 && heads >= 1 && dim % heads == 0,
                "ncf_attention_fwd: bad shape (groups=%lld L=%lld H=%lld D=%lld; L<=64)",
                (long long)groups, (long long)group_len, (long long)heads, (long long)dim);
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_attention_fwd: dropout_p out of [0,1)");
  if (groups == 0) return NCF_OK;
  hipStream_t st = (hipStream_t)stream;
  const int L = (int)group_len, H = (int)heads;
  switch (dim / heads) {
    case 8: return fwd_hd<8>(q, k, v, groups, L, H, dropout_p, seed, clock, probs, out, st, mask);
    case 16: return fwd_hd<16>(q, k, v, groups, L, H, dropout_p, seed, clock, probs, out, st, mask);
    case 32: return fwd_hd<32>(q, k, v, groups, L, H, dropout_p, seed, clock, probs, out, st, mask);
    case 64: return fwd_hd<64>(q, k, v, groups, L, H, dropout_p, seed, clock, probs, out, st, mask);
  }
  ncf_set_error("ncf_attention_fwd: head dim %lld unsupported (8/16/32/64)", (long long)(dim / heads));
  return NCF_ERR_ARG;
}

extern "C" int ncf_attention_fwd(const float* q, const float* k, const float* v, int64_t groups,
                                 int64_t group_len, int64_t heads, int64_t dim, float dropout_p,
                                 uint64_t seed, const ncf_step_clock* clock, float* probs, float* out, void* stream) {
  return attention_fwd(q, k, v, groups, group_len, heads, dim, dropout_p, seed, clock, probs, out,
                       nullptr, stream);
}

extern "C" int ncf_attention_fwd_masked(const float* q, const float* k, const float* v,
                                        int64_t groups, int64_t group_len, int64_t heads,
                                        int64_t dim, float dropout_p, uint64_t seed,
                                        const ncf_step_clock* clock, const uint8_t* mask,
                                        float* probs, float* out, void* stream) {
  NCF_CHECK_ARG(mask != nullptr, "ncf_attention_fwd_masked: NULL mask");
  return attention_fwd(q, k, v, groups, group_len, heads, dim, dropout_p, seed, clock, probs, out,
                       mask, stream);
}

extern "C" int ncf_attention_bwd(const float* q, const float* k, const float* v, const float* probs,
                                 const float* grad_out, int64_t groups, int64_t group_len,
                                 int64_t heads, int64_t dim, float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                                 float* grad_scores, float* grad_q, float* grad_k, float* grad_v,
                                 void* stream) {
  NCF_CHECK_ARG(groups >= 0 && group_len >= 1 && group_len <= 64 && heads >= 1 && dim % heads == 0,
                "ncf_attention_bwd: bad shape");
  if (groups == 0) return NCF_OK;
  hipStream_t st = (hipStream_t)stream;
  const int L = (int)group_len, H = (int)heads;
  switch (dim / heads) {
    case 8: return bwd_hd<8>(q, k, v, probs, grad_out, groups, L, H, dropout_p, seed, clock, grad_scores, grad_q, grad_k, grad_v, st);
    case 16: return bwd_hd<16>(q, k, v, probs, grad_out, groups, L, H, dropout_p, seed, clock, grad_scores, grad_q, grad_k, grad_v, st);
    case 32: return bwd_hd<32>(q, k, v, probs, grad_out, groups, L, H, dropout_p, seed, clock, grad_scores, grad_q, grad_k, grad_v, st);
    case 64: return bwd_hd<64>(q, k, v, probs, grad_out, groups, L, H, dropout_p, seed, clock, grad_scores, grad_q, grad_k, grad_v, st);
  }
  ncf_set_error("ncf_attention_bwd: head dim unsupported");
  return NCF_ERR_ARG;
}
