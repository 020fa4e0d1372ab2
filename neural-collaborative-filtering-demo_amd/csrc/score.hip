// Batch candidate scoring: top-K items for many users over the whole catalogue (C5: 10K users x
// 1M items), the accelerated form of the reference's serving loop
// `model.forward_simple(customer, all_products)` + `nlargest(top_k, 'score')`
// (src/inference/demo/app.py:44-75; forward_simple: src/model/architecture.py:409-485).
//
// Factorised form: in eval with one item per group, softmax over a single key is
// 1, so the MLP path depends on the item only, and
//   logit(u, i) = q_u . p_i + bias_i,  q_u = w0 * LN_mf(U_mf[u]) (.) w_mf,  p_i = LN_mf(I_mf[i]),
//   bias_i = w1 * mlp_item(i) + w0 * b_mf + b_final,     score = sigmoid(logit)  (monotone).
// Pipeline (all deterministic: the final order is (logit desc, item id asc)):
//   1. ncf_score_queries      q_u rows (gather + LayerNorm + scale);
//   2. ncf_score_kth          per user, the K-th largest logit over a strided item SAMPLE (the
//                             sample logits, bias included, come from ncf_gemm_f32 with a strided
//                             B) — a lower bound of the true K-th largest (k_kth_lds: the row in
//                             LDS, two levels of 256 linear value bins; k_kth: radix select over
//                             the order-preserving uint32 image of the float, streamed);
//   3. ncf_score_collect_split  the MFMA scan (k_collect3: bf16 matrix cores on operands split into
//                             bf16 terms; ncf_score_collect: the fp32 MFMA scan), appending
//                             (logit, item) to the user's candidate list when logit >= threshold.
//                             The candidate SET is a function of the threshold only, so any append
//                             order gives the same result.  With one or two terms the scan's
//                             logits are bounds (within E_u = c |q_u| max|p|, c = 8e-3 / 1e-4):
//                             ncf_score_margin lowers the thresholds by E_u first;
//   4. ncf_score_select(_rescored)  per user, radix select of the K-th candidate key in LDS, the K
//                             winners sorted (after 1/2-term scans: the candidates within 2 E_u of
//                             the scan's K-th re-scored in fp32 first); when a user's list
//                             overflowed, the K-th best candidate seen is a higher valid threshold
//                             and the host re-runs 3-4 for those users.  With a rank-j threshold
//                             (j < K, a smaller sample: thr_check) it also checks that the K chosen
//                             are provably the top K, and flags the user for a re-run if not.
// Tilings: see k_collect (fp32) and k_collect3 (split bf16) below.
#include "ncf_common.h"
#include <algorithm>
#include <type_traits>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t fkey(float f) {  // order-preserving float -> uint32
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// ---- 1. queries: q = w0 * LN(U_mf[id]) (.) w_mf; L = D/4 lanes per row.  The rows are QD =
// max(64, D) floats wide: a D < 64 row is zero-padded (the item index pads its rows the same way,
// so every dot product is the D-term one — the scan kernels are 64-deep; D = 128 rows are
// scanned 128-deep by the fp32 scan, k_collect<128>)
template <int D, int kQD = (D > 64 ? D : 64)>
__global__ void k_queries(const int64_t* __restrict__ ids, int64_t n, const float* __restrict__ table,
                          int64_t rows, const float* __restrict__ gamma,
                          const float* __restrict__ beta, float eps,
                          const float* __restrict__ w_mf, const float* __restrict__ final_w,
                          float* __restrict__ q, int* __restrict__ err) {
  constexpr int L = D / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = t / L;
  const int c = (int)(t % L) * 4;
  if (r >= n) return;  // whole row groups retire together (L divides 64)
  int64_t id = ids[r];
  if (id < 0 || id >= rows) {
    if (err && c == 0) atomicOr(err, 1);
    id = 0;
  }
  const float4 x = ld4(table + id * D + c);
  const float mean = group_sum<L>(x.x + x.y + x.z + x.w) * (1.0f / D);
  const float4 xc = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
  const float var = group_sum<L>(xc.x * xc.x + xc.y * xc.y + xc.z * xc.z + xc.w * xc.w) * (1.0f / D);
  const float rstd = 1.0f / sqrtf(var + eps);
  const float4 g = ld4(gamma + c), b = ld4(beta + c), w = ld4(w_mf + c);
  const float w0 = final_w[0];
  st4(q + r * kQD + c, make_float4(w0 * ((xc.x * rstd * g.x + b.x) * w.x),
                                   w0 * ((xc.y * rstd * g.y + b.y) * w.y),
                                   w0 * ((xc.z * rstd * g.z + b.z) * w.z),
                                   w0 * ((xc.w * rstd * g.w + b.w) * w.w)));
#pragma unroll
  for (int pc = D + c; pc < kQD; pc += D) st4(q + r * kQD + pc, make_float4(0.f, 0.f, 0.f, 0.f));
}

// bias_i = w1 * mlp_item_i + (w0 * b_mf + b_final)
__global__ void k_item_bias(const float* __restrict__ mlp_item, int64_t n,
                            const float* __restrict__ final_w, const float* __restrict__ final_b,
                            const float* __restrict__ mf_b, float* __restrict__ bias) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bias[i] = final_w[1] * mlp_item[i] + (final_w[0] * mf_b[0] + final_b[0]);
}

// ---- 2. K-th largest of each row of a [users, S] logit matrix (radix select, 4 x 8-bit digits)
// logit(u, j) = logits[u*S + j] + bias[j * stride] (the sample is every stride-th item)
__global__ __launch_bounds__(256) void k_kth(const float* __restrict__ logits, int64_t S, int K,
                                             const float* __restrict__ bias, int64_t stride,
                                             float* __restrict__ thr) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_need;
  const float* row = logits + (int64_t)blockIdx.x * S;
  uint32_t prefix = 0, need = (uint32_t)(K < S ? K : S);  // rank from the top, 1-based
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
    hist[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t j = threadIdx.x; j < S; j += 256) {
      const uint32_t k = fkey(bias ? row[j] + bias[j * stride] : row[j]);
      if ((k & hmask) == (prefix & hmask)) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // walk digits from the top until the rank is reached
      uint32_t acc = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (acc + hist[d] >= need) break;
        acc += hist[d];
      }
      s_prefix = prefix | ((uint32_t)d << shift);
      s_need = need - acc;
    }
    __syncthreads();
    prefix = s_prefix;
    need = s_need;
    __syncthreads();
  }
  // the sample logits come from a GEMM with another k order than the collect kernel: lower the
  // bound by a margin far above the fp32 reordering error of a 64-term dot product (a lower
  // threshold only admits more candidates, never loses one)
  if (threadIdx.x == 0) {
    const float v = fkey_inv(prefix);
    thr[blockIdx.x] = v - 1e-4f * fmaxf(1.0f, fabsf(v));
  }
}

// The same threshold with the row held in LDS: the logits (+ the sampled bias, a strided gather)
// are read from HBM once, with float4 loads, and the select runs over LDS in value space: 256
// linear bins over [min, max], then 256 sub-bins of the bin holding the K-th largest; the
// threshold is the smallest logit in the sub-bin holding it (at least K sample logits are >= it;
// it is below the exact K-th by less than (max - min) / 65536, far inside the margin).  Linear
// bins spread the logits over many bins (the exponent byte of the radix keys puts nearly all of
// them in one or two, and their LDS atomics serialise).  For S <= kKthLdsMax.
constexpr int64_t kKthLdsMax = 38912;   // 152 KB of logits (of the 160 KB of LDS)

// wave 0: the highest bin d with (count of bins >= d) >= need; returns d, and the count above d
// in *above (lane l holds bins 4l..4l+3)
__device__ __forceinline__ int kth_walk(const uint32_t* hist, uint32_t need, uint32_t* above) {
  const int l = threadIdx.x;
  const uint32_t c0 = hist[4 * l], c1 = hist[4 * l + 1], c2 = hist[4 * l + 2], c3 = hist[4 * l + 3];
  uint32_t suf = c0 + c1 + c2 + c3;   // inclusive suffix over lanes, from the top
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_down(suf, o, 64);
    if (l + o < 64) suf += x;
  }
  const uint64_t m = __ballot(suf >= need);            // lanes 0..L (suffix non-increasing)
  const int L = 63 - __builtin_clzll(m);
  // in lane L: walk its four bins from the top
  uint32_t acc = suf - (c0 + c1 + c2 + c3);
  int j = 3;
  if (acc + c3 < need) {
    acc += c3; j = 2;
    if (acc + c2 < need) {
      acc += c2; j = 1;
      if (acc + c1 < need) { acc += c1; j = 0; }
    }
  }
  *above = __shfl(acc, L, 64);
  return 4 * L + __shfl(j, L, 64);
}

// NT threads: 1024 for long samples (one workgroup per CU: more loads and LDS sweeps in flight),
// 512 for short ones (several workgroups per CU)
// E = float: fp32 sample logits (bias added here when given); E = _Float16: the fp16 logits of
// k_sample16 (bias included, rounded down), kept as fp16 in LDS (2 S bytes: two workgroups per CU
// at S = 38912).  Every comparison is on the widened fp32 value.
template <typename E>
__device__ __forceinline__ float4 ld_logit4(const E* p);
template <>
__device__ __forceinline__ float4 ld_logit4<float>(const float* p) { return ld4(p); }
template <>
__device__ __forceinline__ float4 ld_logit4<_Float16>(const _Float16* p) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 v = *reinterpret_cast<const h4*>(p);
  return make_float4((float)v.x, (float)v.y, (float)v.z, (float)v.w);
}
template <typename E>
__device__ __forceinline__ void st_logit4(E* p, float4 v);
template <>
__device__ __forceinline__ void st_logit4<float>(float* p, float4 v) {
  *reinterpret_cast<float4*>(p) = v;
}
template <>
__device__ __forceinline__ void st_logit4<_Float16>(_Float16* p, float4 v) {   // (exact: v is fp16)
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  *reinterpret_cast<h4*>(p) = h4{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
}

// The bin range [vmin, vmax] spans the FINITE sample values only: an fp16 sample logit below
// -65504 is stored as -inf (rounded toward -inf, k_sample16), and a -inf (or a NaN) in the range
// would make its scale 0 / NaN and every value fall into bin 0.  Non-finite values clamp into
// bin 0 (below the range; a +inf cannot occur: the rounding saturates at 65504), so the
// threshold stays a valid lower bound whatever the sample holds.
__device__ __forceinline__ float fin_lo(float x) { return __builtin_isfinite(x) ? x : -INFINITY; }
__device__ __forceinline__ float fin_hi(float x) { return __builtin_isfinite(x) ? x : INFINITY; }

template <int NT, typename E = float>
__global__ __launch_bounds__(NT) void k_kth_lds(const E* __restrict__ logits, int64_t S,
                                                 int K, const float* __restrict__ bias,
                                                 int64_t stride, float* __restrict__ thr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char kth_raw[];
  E* kth_vals = reinterpret_cast<E*>(kth_raw);
  __shared__ uint32_t hist[256], hmin[256];
  __shared__ float rmax[NT / 64], rmin[NT / 64];
  __shared__ int s_bin;
  __shared__ uint32_t s_need;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const E* row = logits + (int64_t)blockIdx.x * S;
  float vmax = -INFINITY, vmin = INFINITY;
  const int64_t S4 = (S & 3) == 0 ? S / 4 : 0;   // rows start 4-element aligned when S % 4 == 0
  // 4 float4 loads in flight per thread (a dependent load per iteration leaves the row's HBM
  // latency exposed 15 times at S = 30720)
  for (int64_t base = tid; base < S4; base += 4 * NT) {
    float4 xs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j4 = base + (int64_t)u * NT;
      xs[u] = j4 < S4 ? ld_logit4<E>(row + 4 * j4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j4 = base + (int64_t)u * NT;
      if (j4 >= S4) break;
      const float4 x = xs[u];
      const int64_t j = 4 * j4;
      const float4 v = bias ? make_float4(x.x + bias[j * stride], x.y + bias[(j + 1) * stride],
                                          x.z + bias[(j + 2) * stride],
                                          x.w + bias[(j + 3) * stride])
                            : x;
      st_logit4<E>(kth_vals + j, v);
      vmax = fmaxf(vmax, fmaxf(fmaxf(fin_lo(v.x), fin_lo(v.y)), fmaxf(fin_lo(v.z), fin_lo(v.w))));
      vmin = fminf(vmin, fminf(fminf(fin_hi(v.x), fin_hi(v.y)), fminf(fin_hi(v.z), fin_hi(v.w))));
    }
  }
  for (int64_t j = 4 * S4 + tid; j < S; j += NT) {
    const float v = bias ? (float)row[j] + bias[j * stride] : (float)row[j];
    kth_vals[j] = (E)v;
    vmax = fmaxf(vmax, fin_lo(v));
    vmin = fminf(vmin, fin_hi(v));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    vmax = fmaxf(vmax, __shfl_xor(vmax, o, 64));
    vmin = fminf(vmin, __shfl_xor(vmin, o, 64));
  }
  if (lane == 0) { rmax[w] = vmax; rmin[w] = vmin; }
  for (int j = tid; j < 256; j += NT) { hist[j] = 0; hmin[j] = 0xFFFFFFFFu; }
  __syncthreads();
  vmax = rmax[0]; vmin = rmin[0];
#pragma unroll
  for (int k = 1; k < NT / 64; ++k) { vmax = fmaxf(vmax, rmax[k]); vmin = fminf(vmin, rmin[k]); }
  const uint32_t need0 = (uint32_t)(K < S ? K : S);   // rank from the top, 1-based
  float v = vmax;
  if (vmax > vmin) {
    // level 0: 256 bins over [vmin, vmax]; b(v) is non-decreasing in v
    const float inv0 = 256.0f / (vmax - vmin);
    auto bin0 = [&](float x) { return (int)fminf(fmaxf((x - vmin) * inv0, 0.0f), 255.0f); };
    for (int64_t j = tid; j < S; j += NT) atomicAdd(&hist[bin0((float)kth_vals[j])], 1u);
    __syncthreads();
    if (w == 0) {
      uint32_t above = 0;
      const int b = kth_walk(hist, need0, &above);
      if (lane == 0) {
        s_bin = b;
        s_need = need0 - above;
      }
    }
    __syncthreads();
    const int b0 = s_bin;
    const uint32_t need1 = s_need;
    for (int j = tid; j < 256; j += NT) hist[j] = 0;
    __syncthreads();
    // level 1: 256 sub-bins of bin b0, with the smallest logit of each (as an order key)
    const float lo1 = vmin + (float)b0 / inv0, inv1 = inv0 * 256.0f;
    for (int64_t j = tid; j < S; j += NT) {
      const float x = (float)kth_vals[j];
      if (bin0(x) == b0) {
        const int sb = (int)fminf(fmaxf((x - lo1) * inv1, 0.0f), 255.0f);
        atomicAdd(&hist[sb], 1u);
        atomicMin(&hmin[sb], fkey(x));
      }
    }
    __syncthreads();
    if (w == 0) {
      uint32_t above = 0;
      const int b1 = kth_walk(hist, need1, &above);
      if (lane == 0) s_bin = b1;
    }
    __syncthreads();
    v = fkey_inv(hmin[s_bin]);
  }
  if (tid == 0) thr[blockIdx.x] = v - 1e-4f * fmaxf(1.0f, fabsf(v));   // (the margin of k_kth)
}

// max_i ||p_i||_2 over the item rows (D = 64).  Grid-stride: a 16-lane group reads one row
// (a float4 per lane) per iteration and keeps its running max of the squared norm; the block
// reduces that in LDS and issues ONE integer atomicMax (non-negative floats order like their
// bit patterns).  (Was: one atomicMax per row into the same address — 1M same-address atomics,
// 11 ms for a 256 MB table.)
constexpr int kNormMaxBlocks = 1024;
__global__ __launch_bounds__(256) void k_row_norm_max(const float* __restrict__ p, int64_t n,
                                                      uint32_t* __restrict__ out_bits) {
  __shared__ float s_max[4];
  const int sub = threadIdx.x & 15;
  const int64_t grp0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int64_t ngrp = ((int64_t)gridDim.x * 256) >> 4;
  float best = 0.0f;
  for (int64_t row = grp0; row < n; row += ngrp) {     // (a group's 16 lanes agree on `row`)
    const float4 x = reinterpret_cast<const float4*>(p + row * 64)[sub];
    float ss = x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
    best = fmaxf(best, ss);
  }
  best = fmaxf(best, __shfl_xor(best, 16, 64));
  best = fmaxf(best, __shfl_xor(best, 32, 64));
  if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
    atomicMax(out_bits, __float_as_uint(sqrtf(m)));
  }
}

// thr[u] -= c * ||q_u||_2 * max_i ||p_i||_2 (+ an ulp-scale allowance): the two-term split
// scan's logits are within that of the fp32 logit (Cauchy-Schwarz over the dropped terms), so
// the lowered threshold keeps every item the fp32 threshold would
__global__ __launch_bounds__(256) void k_score_margin(const float* __restrict__ q,
                                                      const int32_t* __restrict__ user_list,
                                                      int64_t n, const uint32_t* __restrict__ pmax,
                                                      float c, float* __restrict__ thr) {
  const int64_t slot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (slot >= n) return;
  const int64_t u = user_list ? (int64_t)user_list[slot] : slot;
  const float x = q[u * 64 + lane];
  float ss = x * x;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if (lane == 0) {
    const float t = thr[u];
    const float e = c * sqrtf(ss) * __uint_as_float(*pmax);
    thr[u] = t - (e * 1.0001f + 1e-6f * fabsf(t));
  }
}

// ---- 3. MFMA scan + threshold filter
// fp32 tiling (k_collect): a 512-thread workgroup owns 256 users (8 waves x 32), keeps each
// wave's q rows in registers (k-permuted: MFMA step s uses k = s + (D/2)h), and streams 32-item
// tiles of p through double-buffered LDS ([32][D+1] pitch: conflict-free); per tile a wave issues
// D/2 v_mfma_f32_32x32x2_f32 and filters its 32x32 logits against 16 per-lane thresholds (D = 64,
// or 128: the C4 model's width, two k chunks per tile).  Hits are
// staged in LDS (one LDS atomic per wave and tile) and flushed to the global per-user lists in
// parallel bursts (a global atomic per hit made the wave wait thousands of cycles per tile).
constexpr int kUsersPerBlock = 256;  // 8 waves x 32
constexpr int kItemTile = 32;
#ifndef NCF_SCORE_PD
#define NCF_SCORE_PD 1
#endif
constexpr int kPD = NCF_SCORE_PD;     // item tiles in flight (register ring)
constexpr int kCandBuf = 2048;        // LDS-staged candidates per workgroup (flushed at half)

template <int D>
__global__ __launch_bounds__(512) void k_collect(
    const float* __restrict__ q, const int32_t* __restrict__ user_list, int64_t n_users,
    const float* __restrict__ items, const float* __restrict__ bias, int64_t n_items,
    int64_t items_per_block, const float* __restrict__ thr, int64_t cap,
    uint32_t* __restrict__ count, ncf_score_cand* __restrict__ cand) {
  static_assert(D == 64 || D == 128, "the fp32 scan takes 64- or 128-deep rows");
  constexpr int KH = D / 2;      // k per lane half (MFMA step s: k = s + KH h)
  constexpr int NV = D / 64;     // float4 per thread to stage a 32 x D tile
  __shared__ float ps[2][kItemTile][D + 1];
  __shared__ float bs[2][kItemTile];
  // Candidates are staged in LDS (an LDS atomic returns in ~100 cycles; a global one in
  // thousands, and a wave waits for it in the filter of nearly every tile) and flushed to the
  // per-user global lists in parallel bursts.  The lists are sets (select sorts them), so the
  // staging order does not matter.
  __shared__ float cl[kCandBuf];
  __shared__ int32_t ci[kCandBuf], cu[kCandBuf];
  __shared__ uint32_t ccount;
  if (threadIdx.x == 0) ccount = 0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  // this wave's 32 users (slot = index into the user list)
  const int64_t slot0 = (int64_t)blockIdx.y * kUsersPerBlock + w * 32;
  const int64_t my_slot = slot0 + i;
  const bool uvalid = my_slot < n_users;
  const int64_t my_user = uvalid ? (user_list ? user_list[my_slot] : my_slot) : 0;
  float a[KH];
  {
    const float* qp = q + my_user * D + KH * h;
#pragma unroll
    for (int v = 0; v < KH / 4; ++v) {
      const float4 x = ld4(qp + 4 * v);
      a[4 * v] = x.x; a[4 * v + 1] = x.y; a[4 * v + 2] = x.z; a[4 * v + 3] = x.w;
    }
  }
  // Consume the query registers here: with their loads still pending at the loop header the
  // compiler's wait-count pass puts a vmcnt(0) in front of their first MFMA in EVERY
  // iteration, which also drains the next tile's prefetch and exposes its HBM latency (measured:
  // the matrix cores idle half the time).
#pragma unroll
  for (int k = 0; k < KH; ++k) asm volatile("" ::"v"(a[k]));
  // thresholds of the 16 users whose logits this lane holds: row (r&3) + 8(r>>2) + 4h
  float th[16];
  int64_t urow[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = slot0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    const bool v = s < n_users;
    urow[r] = v ? (user_list ? user_list[s] : s) : -1;
    th[r] = v ? thr[urow[r]] : INFINITY;
  }
  const int64_t it0 = (int64_t)blockIdx.x * items_per_block;
  const int64_t it1 = min(n_items, it0 + items_per_block);
  // staging: 512 threads x NV float4 = one 32 x D tile
  const int sj = tid >> 4, sk = (tid & 15) * 4;
  auto fetch = [&](int64_t t0, float4 (&v)[NV], float& bv) {
    const int64_t item = t0 + sj;
    const int64_t src = item < it1 ? item : it0;  // clamped, unconditional
#pragma unroll
    for (int c = 0; c < NV; ++c) v[c] = ld4(items + src * D + sk + 64 * c);
    bv = bias[src];
  };
  // register ring of kPD staged tiles: the load of tile t + kPD is issued while tile t is
  // multiplied, so a tile's HBM latency hides behind kPD tiles of MFMAs (one tile alone,
  // ~2K cycles per wave, is shorter than a loaded HBM miss)
  float4 pv[kPD][NV];
  float pb[kPD];
#pragma unroll
  for (int d = 0; d < kPD; ++d)
    if (it0 + d * kItemTile < it1) fetch(it0 + d * kItemTile, pv[d], pb[d]);
  int buf = 0, slot = 0;
  auto flush = [&](uint32_t nstaged) {
    const uint32_t m = nstaged < (uint32_t)kCandBuf ? nstaged : (uint32_t)kCandBuf;
    for (uint32_t e = threadIdx.x; e < m; e += blockDim.x) {
      const int32_t u = cu[e];
      const uint32_t pos = atomicAdd(&count[u], 1u);
      if (pos < cap) cand[(int64_t)u * cap + pos] = ncf_score_cand{cl[e], ci[e]};
    }
  };
  for (int64_t t0 = it0; t0 < it1; t0 += kItemTile) {
    float4 cur[NV];
    float cb = pb[0];
#pragma unroll
    for (int c = 0; c < NV; ++c) cur[c] = pv[0][c];
#pragma unroll
    for (int d = 1; d < kPD; ++d)   // (static slot selection: the ring rotates by one)
      if (slot == d) {
#pragma unroll
        for (int c = 0; c < NV; ++c) cur[c] = pv[d][c];
        cb = pb[d];
      }
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      float* dst = &ps[buf][sj][sk + 64 * c];
      dst[0] = cur[c].x; dst[1] = cur[c].y; dst[2] = cur[c].z; dst[3] = cur[c].w;
    }
    if ((tid & 15) == 0) bs[buf][sj] = cb;
    __syncthreads();
    {
      const uint32_t staged = ccount;     // uniform: read after the barrier
      if (staged >= (uint32_t)kCandBuf / 2) {
        flush(staged);
        __syncthreads();
        if (threadIdx.x == 0) ccount = 0;
        __syncthreads();
      }
    }
    if (t0 + kPD * kItemTile < it1) {
#pragma unroll
      for (int d = 0; d < kPD; ++d)
        if (slot == d) fetch(t0 + kPD * kItemTile, pv[d], pb[d]);
    }
    slot = slot + 1 == kPD ? 0 : slot + 1;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    const float* pb_row = &ps[buf][i][KH * h];
#pragma unroll
    for (int s = 0; s < KH; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], pb_row[s], acc, 0, 0, 0);
    const int64_t item = t0 + i;
    const float b = bs[buf][i];
    const bool ivalid = item < it1;
    uint32_t hm = 0;   // this lane's hits of the tile (bit r: user row r)
#pragma unroll
    for (int r = 0; r < 16; ++r) hm |= (ivalid && acc[r] + b >= th[r]) ? (1u << r) : 0u;
    if (__ballot(hm != 0)) {   // wave-uniform; hits are rare (~1 per wave and tile)
      // one LDS atomic per wave: exclusive prefix of the lanes' hit counts
      const uint32_t nh = (uint32_t)__popc(hm);
      uint32_t incl = nh;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o, 64);
        if (lane >= o) incl += x;
      }
      uint32_t base = 0;
      if (lane == 63) base = atomicAdd(&ccount, incl);
      base = __shfl(base, 63, 64) + incl - nh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (hm & (1u << r)) {
          const float lg = acc[r] + b;
          if (base < (uint32_t)kCandBuf) {
            cl[base] = lg;
            ci[base] = (int32_t)item;
            cu[base] = (int32_t)urow[r];
          } else {   // staging full within this tile: straight to the global list
            const uint32_t pos = atomicAdd(&count[urow[r]], 1u);
            if (pos < cap) cand[urow[r] * cap + pos] = ncf_score_cand{lg, (int32_t)item};
          }
          ++base;
        }
      }
    }
    buf ^= 1;
  }
  __syncthreads();
  flush(ccount);
}

// ---- 3'. the same scan on bf16 matrix cores with fp32 accuracy.  Every operand is split into
// three bf16 terms, x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1):
// 24 significant bits, the fp32 significand), and a logit is the fp32 accumulation of the six
// products whose order is >= 2^-24 relative, a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0
// (v_mfma_f32_32x32x16_bf16: each bf16 x bf16 product is exact in fp32).  The dropped terms are
// below 2^-26 of a product, so a logit differs from the fp32 MFMA scan's by fp32 rounding of
// the accumulation only — far inside the threshold's 1e-4 relative margin (k_kth), so the
// candidate set is unchanged.  6 bf16 MFMAs (32 cycles each) replace 32 fp32 ones (64 cycles)
// per 32 x 32 x 64 tile.  The item rows are split once per index (k_split3: three bf16 planes).
// T = 2 keeps a0 b0 + a0 b1 + a1 b0 (error ~6e-5 |q| max|p|), T = 1 only a0 b0 (bf16 keeps 8
// significant bits: |a0 b0 - a b| <= (2^-7 + 2^-16) |a| |b|, so E = 8e-3 |q| max|p|): both
// lower the thresholds by E and re-score the candidates near the K-th in fp32 (k_select<true>),
// so the top-k do not depend on T.  One product per 32 x 32 x 16 step instead of three: the
// scan went 3.6 -> 2.1 ms at 10K x 1M (it is then no longer MFMA-issue-bound).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(float x, __bf16& x0, __bf16& x1, __bf16& x2) {
  x0 = (__bf16)x;
  const float r1 = x - (float)x0;
  x1 = (__bf16)r1;
  x2 = (__bf16)(r1 - (float)x1);
}

__global__ void k_split3(const float* __restrict__ p, int64_t n, uint16_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  __bf16 x0, x1, x2;
  split3(p[e], x0, x1, x2);
  out[e] = __builtin_bit_cast(uint16_t, x0);
  out[n + e] = __builtin_bit_cast(uint16_t, x1);
  out[2 * n + e] = __builtin_bit_cast(uint16_t, x2);
}

constexpr int kP3 = 72;        // LDS pitch of a staged bf16 item row (64 + 8)
// 32-user blocks per wave: 4 with two-term operands (each staged B operand feeds four MFMA
// chains; 256 VGPRs, no spill), 2 with three terms (their query registers take 1.5x as many)
#ifndef NCF_SCORE3_UB
#define NCF_SCORE3_UB 4
#endif
constexpr int kUB3 = NCF_SCORE3_UB;            // (two-term scan)
constexpr int kUB3t = NCF_SCORE3_UB > 2 ? 2 : NCF_SCORE3_UB;   // (three-term scan)
#ifndef NCF_SCORE3_NW
#define NCF_SCORE3_NW 8
#endif
constexpr int kNW3 = NCF_SCORE3_NW;
#ifndef NCF_SCAN_NB
#define NCF_SCAN_NB 0
#endif
// the one-term scan without the per-tile barrier: measured no faster (graphed top-10 2.33 / 2.34
// against 2.31 / 2.32 ms; scan 1.89-1.91 against 1.86-1.87 ms, r5zi) — the waits it removes were
// on LDS bandwidth (the per-tile threshold and operand reads), not on the barrier itself
constexpr bool kScanNB = NCF_SCAN_NB != 0;
#ifndef NCF_SCAN_MINTH
#define NCF_SCAN_MINTH 1
#endif
constexpr bool kScanMinTh = NCF_SCAN_MINTH != 0;   // the register-only first reject (k_collect3)   // waves per workgroup (measured: 8 at one per CU 6.6 ms, 4 at two per CU 6.9)
// Candidates staged per wave (its own LDS slice, dynamic LDS).  A full slice is written out
// grouped by user: one global counter atomic per (user, flush) and each user's entries stored
// contiguously, instead of one atomic and two scattered 4-byte stores per candidate (measured
// before: 1.17 GB of writes per scan launch for ~0.14 GB of candidates).
// (two-term scan: 1024 entries per wave; three-term: 896, its three tile planes take more of
// the 160 KB)
template <int T>
constexpr int slice3() { return T == 3 ? 896 : 1024; }
// per wave: logit f32 | item i32 | local user u16 | rank u16 | perm u16 [slice3], then
// count / offset / base u32 [32 UB]
template <int UB, int T>
constexpr size_t slice3_bytes() {
  return (size_t)slice3<T>() * (4 + 4 + 2 + 2 + 2) + 3 * 4 * 32 * UB;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));

// One workgroup = 8 waves x 32 users (two waves per SIMD) scanning one item split in 32-item
// tiles.  Per tile, a wave runs 4 steps x 6 bf16 MFMAs into one 32 x 32 accumulator, then
// filters it against its users' thresholds.  Three LDS tile buffers and one barrier per tile; the
// B operands of tile t + 1 are read from LDS while tile t is multiplied.  Hits go to the wave's
// own LDS slice (offsets from ballots, no atomics) and the wave writes its slice to the global
// lists itself when it fills (no workgroup barrier).
// LDS writes of this wave visible to its other lanes (LDS-only fence: no global cache traffic)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// A wave's staged candidates written out grouped by user (k_collect3): per-user counts and
// ranks (LDS atomics), a wave scan for the group offsets, ONE global counter atomic per user
// with candidates, then the entries stored in user-grouped order, consecutive lanes writing
// consecutive slots of a user's list.  Only after the scan loop (inside it, or called out of
// line from it, it pushed the loop's arrays to scratch: 40 GB of scratch writes per launch).
template <int NU>
__device__ __forceinline__ void flush_grouped(
    uint32_t staged, int64_t slot0, const int32_t* __restrict__ user_list,
    uint32_t* __restrict__ count, int64_t cap, ncf_score_cand* __restrict__ cand,
    const float* wl, const int32_t* wi, const uint16_t* wu,
    uint16_t* wr, uint16_t* wp, uint32_t* ucnt, uint32_t* uoff, uint32_t* ubase) {
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < NU; k += 64) ucnt[k] = 0u;
  wave_lds_sync();
  for (uint32_t e = lane; e < staged; e += 64) wr[e] = (uint16_t)atomicAdd(&ucnt[wu[e]], 1u);
  wave_lds_sync();
  // per user: one reservation in its global list; offsets of the user groups in the slice
  uint32_t run = 0;
  for (int c = 0; c < NU / 64; ++c) {
    const int k = 64 * c + lane;
    const uint32_t n = ucnt[k];
    uint32_t incl = n;   // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    uoff[k] = run + incl - n;
    run += __shfl(incl, 63, 64);
    uint32_t b = 0;
    if (n) {
      const int64_t s = slot0 + k;
      b = atomicAdd(&count[user_list ? (int64_t)user_list[s] : s], n);
    }
    ubase[k] = b;
  }
  wave_lds_sync();
  for (uint32_t e = lane; e < staged; e += 64) wp[uoff[wu[e]] + wr[e]] = (uint16_t)e;
  wave_lds_sync();
  for (uint32_t q = lane; q < staged; q += 64) {
    const uint32_t e = wp[q], k = wu[e];
    const uint32_t pos = ubase[k] + (q - uoff[k]);
    if (pos < cap) {
      const int64_t s = slot0 + k;
      const int64_t u = user_list ? (int64_t)user_list[s] : s;
      cand[u * cap + pos] = ncf_score_cand{wl[e], wi[e]};
    }
  }
  wave_lds_sync();
}

// NB (one-term scan only): no shared item tiles and no workgroup barrier — every wave loads its
// own B operands (the 32 items' 16-byte fragments of each MFMA step) straight into registers, one
// tile ahead, and runs at its own pace; the eight waves of a workgroup read the same item lines,
// which L1 / L2 serve.  (The shared-tile form parks each wave at the per-tile barrier until the
// slowest wave's filter is done: 38% of the wave time at top-10, r4h SQ counters.)
template <int UB, int NW, int T, bool NB = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void k_collect3(
    const float* __restrict__ q, const int32_t* __restrict__ user_list, int64_t n_users,
    const uint16_t* __restrict__ items3, const float* __restrict__ bias, int64_t n_items,
    int64_t items_per_block, int ub, const float* __restrict__ thr, int64_t cap,
    uint32_t* __restrict__ count, ncf_score_cand* __restrict__ cand) {
  constexpr int D = 64;
  __shared__ __attribute__((aligned(16))) uint16_t ps[3][T][kItemTile][kP3];
  __shared__ float bs[3][kItemTile];
  extern __shared__ __attribute__((aligned(16))) unsigned char slices3[];
  // consecutive workgroups go round-robin to the 8 XCDs (each with its own L2): give every XCD a
  // contiguous run of the split-major order, so the user blocks of one item split share an L2
  int M = (int)blockIdx.x;
  {
    const int per = (int)(gridDim.x / 8);
    if (per > 0 && (int)blockIdx.x < 8 * per) M = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  }
  const int bx = M / ub, by = M % ub;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  // the wave's UB blocks of 32 users (UB = 2: every staged B operand feeds two MFMA chains)
  const int64_t slot0 = (int64_t)by * (32 * NW * UB) + w * (32 * UB);
  // this lane's query values q[user][32h + 8t + j] split into three bf16 terms, per MFMA step t
  bf16x8_t a0[UB][4], a1[UB][4], a2[UB][4];
#pragma unroll
  for (int ub = 0; ub < UB; ++ub) {
    const int64_t my_slot = slot0 + 32 * ub + i;
    const int64_t my_user = my_slot < n_users ? (user_list ? user_list[my_slot] : my_slot) : 0;
    const float* qp = q + my_user * D + 32 * h;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 x = ld4(qp + 8 * t), y = ld4(qp + 8 * t + 4);
      const float v[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 b0, b1, b2;
        split3(v[j], b0, b1, b2);
        a0[ub][t][j] = b0; a1[ub][t][j] = b1; a2[ub][t][j] = b2;
      }
    }
  }
  // the 16 users whose logits this lane holds: rows (r&3) + 8(r>>2) + 4h of each user block
  // (their ids are looked up at the flush only: 32 fewer live registers in the loop)
  // thresholds of the wave's users in LDS (in registers they would cost 16 VGPRs per user block)
  __shared__ __attribute__((aligned(16))) float ths[NW * 32 * UB];
  float* wth = ths + w * (32 * UB);
#pragma unroll
  for (int ub = 0; ub < UB; ++ub) {
    const int64_t s = slot0 + 32 * ub + i;
    const float v = s < n_users ? thr[user_list ? (int64_t)user_list[s] : s] : INFINITY;
    if (h == 0) wth[32 * ub + i] = v;
  }
  // this lane's 16 thresholds of user block ub: rows (r&3) + 8(r>>2) + 4h, four float4 reads
  auto th_of = [&](int ub, float (&t)[16]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 x = *reinterpret_cast<const float4*>(wth + 32 * ub + 8 * c + 4 * h);
      t[4 * c] = x.x; t[4 * c + 1] = x.y; t[4 * c + 2] = x.z; t[4 * c + 3] = x.w;
    }
  };
  // (kScanMinTh) the smallest threshold of the 16 users each lane's rows hold, per user block
  float thmin[UB];
  if constexpr (kScanMinTh) {
    wave_lds_sync();
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      float t[16];
      th_of(ub, t);
      float m = t[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) m = fminf(m, t[r]);
      thmin[ub] = m;
    }
  }
  const int64_t it0 = (int64_t)bx * items_per_block;
  const int64_t it1 = min(n_items, it0 + items_per_block);
  // staging: thread (item sj, column group sk) holds 4 bf16 of each of the 3 planes of the next
  // tile to store (a one-tile register ring: its load has a whole tile to land)
  constexpr int E = kItemTile * 64 / (64 * NW);   // bf16 per plane per thread: 4 or 8
  using V = typename std::conditional<E == 8, uint4, uint2>::type;
  const int sj = tid / (64 / E), sk = (tid % (64 / E)) * E;
  V pv[T];
  float pb = 0.f;
  // (two planes, 8 waves: each thread stages 8 bf16 of ONE plane with one 16-B load and store)
  constexpr bool ONE = T == 2 && NW == 8;   // (measured: scan 3.64-3.68 -> 3.62-3.64 ms)
  const int pl1 = tid >> 8, sj1 = (tid & 255) >> 3, sk1 = (tid & 7) * 8;
  uint4 pv1;
  auto fetch = [&](int64_t t0) {
    if constexpr (ONE) {
      const int64_t item = t0 + sj1;
      const int64_t src = item < it1 ? item : it0;  // clamped, unconditional
      pv1 = *reinterpret_cast<const uint4*>(items3 + (int64_t)pl1 * n_items * D + src * D + sk1);
      if (pl1 == 0 && sk1 == 0) pb = bias[src];
    } else {
      const int64_t item = t0 + sj;
      const int64_t src = item < it1 ? item : it0;  // clamped, unconditional
#pragma unroll
      for (int pl = 0; pl < T; ++pl)
        pv[pl] = *reinterpret_cast<const V*>(items3 + (int64_t)pl * n_items * D + src * D + sk);
      pb = bias[src];
    }
  };
  auto put = [&](int bb) {
    if constexpr (ONE) {
      *reinterpret_cast<uint4*>(&ps[bb][pl1][sj1][sk1]) = pv1;
      if (pl1 == 0 && sk1 == 0) bs[bb][sj1] = pb;
    } else {
#pragma unroll
      for (int pl = 0; pl < T; ++pl) *reinterpret_cast<V*>(&ps[bb][pl][sj][sk]) = pv[pl];
      if (sk == 0) bs[bb][sj] = pb;
    }
  };
  bf16x8_t bq[UB == 1 ? 4 : 1][3];   // (UB = 1) B operands of the tile being multiplied
  auto rd = [&](int bb, int t) {
#pragma unroll
    for (int pl = 0; pl < T; ++pl)
      bq[UB == 1 ? t : 0][pl] = *reinterpret_cast<const bf16x8_t*>(&ps[bb][pl][i][32 * h + 8 * t]);
  };
  // the wave's candidate slice: staged entries (wave-uniform), written out when it would overflow
  constexpr int NU = 32 * UB;   // the wave's users (local index: 32 ub + row)
  constexpr int kSlice3 = slice3<T>();
  unsigned char* sb = slices3 + (size_t)w * slice3_bytes<UB, T>();
  float* wl = reinterpret_cast<float*>(sb);
  int32_t* wi = reinterpret_cast<int32_t*>(sb + 4 * kSlice3);
  uint16_t* wu = reinterpret_cast<uint16_t*>(sb + 8 * kSlice3);
  uint16_t* wr = wu + kSlice3;       // rank of an entry among its user's
  uint16_t* wp = wr + kSlice3;       // entry of each user-grouped position
  uint32_t* ucnt = reinterpret_cast<uint32_t*>(sb + 14 * kSlice3);
  uint32_t* uoff = ucnt + NU;
  uint32_t* ubase = uoff + NU;
  uint32_t staged = 0;
  // a slice that fills inside the scan loop is written out one candidate at a time (one counter
  // atomic each: what the loop's register budget allows); the rest, grouped after the loop
  auto wflush = [&]() {
    for (uint32_t e = lane; e < staged; e += 64) {
      const int64_t sl = slot0 + wu[e];
      const int64_t u = user_list ? (int64_t)user_list[sl] : sl;
      const uint32_t pos = atomicAdd(&count[u], 1u);
      if (pos < cap) cand[u * cap + pos] = ncf_score_cand{wl[e], wi[e]};
    }
    staged = 0;
  };
  auto filt = [&](const f32x16& acc, int ub, float b, int64_t t0) {
    const int32_t item = (int32_t)(t0 + i);
    if constexpr (kScanMinTh) {
      // Weakest test first, from registers: the lane's largest logit against the smallest of its
      // 16 users' thresholds.  Exact, no margin: a row the exact test accepts has
      // fl(acc[r] + b) >= th[r] >= thmin, and fl(max acc + b) >= fl(acc[r] + b) (rounding is
      // monotone).  Only tiles it passes read the 16 thresholds from LDS.
      f32x2 mx = {acc[0], acc[1]};
#pragma unroll
      for (int r = 2; r < 16; r += 2) mx = __builtin_elementwise_max(mx, f32x2{acc[r], acc[r + 1]});
      if (!__ballot(t0 + i < it1 && fmaxf(mx.x, mx.y) + b >= thmin[ub])) return;
    }
    float th[16];
    th_of(ub, th);
    const bool ivalid = t0 + i < it1;
    // Cheap reject first: max_r (acc[r] - th[r]) + b on packed fp32 (8 v_pk_add + 8 max).  The
    // margin keeps every lane the exact test below could accept (they round differently by at
    // most an ulp of |b|; the subtraction near a hit is exact, Sterbenz).  (Keeping the maximum
    // per group of 4 rows and testing rows only in the groups that pass measured slower: scan
    // 2.19 against 2.05 ms at top-10.)
    {
      f32x2 m2 = {-INFINITY, -INFINITY};
#pragma unroll
      for (int r = 0; r < 16; r += 2)
        m2 = __builtin_elementwise_max(m2, f32x2{acc[r], acc[r + 1]} - f32x2{th[r], th[r + 1]});
      const bool near = ivalid && fmaxf(m2.x, m2.y) + b >= -1e-6f * fabsf(b);
      if (!__ballot(near)) return;
    }
    // exact hits row by row: one wave mask per user row, slice offsets from mbcnt; the slice is
    // written out first when the row's hits would not fit (a row has at most 64)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint64_t hm = __ballot(ivalid && acc[r] + b >= th[r]);
      if (hm == 0) continue;   // wave-uniform
      const uint32_t nh = (uint32_t)__popcll(hm);
      if (staged + nh > (uint32_t)kSlice3) wflush();
      if ((hm >> lane) & 1) {
        const uint32_t at = staged + __builtin_amdgcn_mbcnt_hi(
            (uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
        wl[at] = acc[r] + b;
        wi[at] = item;
        wu[at] = (uint16_t)(32 * ub + (r & 3) + 8 * (r >> 2) + 4 * h);   // local user slot
      }
      staged += nh;
    }
  };
  // Iteration t multiplies tile t (buffer t % 3, operands in registers, the reads of tile t + 1
  // issued behind each step's MFMAs), filters it, stores tile t + 2 into buffer (t + 2) % 3 (it
  // held tile t - 1, whose reads completed before the previous barrier), loads tile t + 3 into
  // the ring, and ends at the barrier that publishes tile t + 2.
  if constexpr (NB) {
    static_assert(T == 1, "the barrier-free scan is the one-term scan");
    wave_lds_sync();   // (this wave's thresholds, written above)
    if (it0 < it1) {
      uint4 bcur[4], bnxt[4];
      float bcur_b = 0.f, bnxt_b = 0.f;
      auto gload = [&](int64_t t0, uint4 (&v)[4], float& bb) {
        const int64_t item = t0 + i;
        const int64_t src = item < it1 ? item : it0;   // clamped, unconditional
        const uint16_t* base = items3 + src * D + 32 * h;
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = *reinterpret_cast<const uint4*>(base + 8 * t);
        bb = bias[src];
      };
      gload(it0, bcur, bcur_b);
      for (int64_t t0 = it0; t0 < it1; t0 += kItemTile) {
        if (t0 + kItemTile < it1) gload(t0 + kItemTile, bnxt, bnxt_b);
        f32x16 acc[UB];
#pragma unroll
        for (int ub = 0; ub < UB; ++ub)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[ub][r] = 0.0f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8_t b0 = __builtin_bit_cast(bf16x8_t, bcur[t]);
#pragma unroll
          for (int ub = 0; ub < UB; ++ub)
            acc[ub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ub][t], b0, acc[ub], 0, 0, 0);
        }
#pragma unroll
        for (int ub = 0; ub < UB; ++ub) filt(acc[ub], ub, bcur_b, t0);
#pragma unroll
        for (int t = 0; t < 4; ++t) bcur[t] = bnxt[t];
        bcur_b = bnxt_b;
      }
    }
  } else if (it0 < it1) {
    fetch(it0);
    put(0);
    if (it0 + kItemTile < it1) {
      fetch(it0 + kItemTile);
      put(1);
    }
    if (it0 + 2 * kItemTile < it1) fetch(it0 + 2 * kItemTile);
    __syncthreads();
    if constexpr (UB == 1) {
#pragma unroll
      for (int t = 0; t < 4; ++t) rd(0, t);
    }
    int bc = 0;
    for (int64_t t0 = it0; t0 < it1; t0 += kItemTile) {
      const int bn = bc == 2 ? 0 : bc + 1, bn2 = bn == 2 ? 0 : bn + 1;
      const bool has_next = t0 + kItemTile < it1;
      f32x16 acc[UB];
#pragma unroll
      for (int ub = 0; ub < UB; ++ub)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[ub][r] = 0.0f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8_t b0, b1, b2;
        if constexpr (UB == 1) {
          b0 = bq[t][0]; b1 = bq[t][T > 1 ? 1 : 0]; b2 = bq[t][T - 1];
        } else {
          b0 = *reinterpret_cast<const bf16x8_t*>(&ps[bc][0][i][32 * h + 8 * t]);
          if constexpr (T >= 2)
            b1 = *reinterpret_cast<const bf16x8_t*>(&ps[bc][1][i][32 * h + 8 * t]);
          if constexpr (T == 3)
            b2 = *reinterpret_cast<const bf16x8_t*>(&ps[bc][T - 1][i][32 * h + 8 * t]);
        }
#pragma unroll
        for (int ub = 0; ub < UB; ++ub) {
          f32x16& c = acc[ub];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ub][t], b0, c, 0, 0, 0);
          if constexpr (T >= 2) {
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ub][t], b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[ub][t], b0, c, 0, 0, 0);
          }
          if constexpr (T == 3) {
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ub][t], b2, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[ub][t], b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[ub][t], b0, c, 0, 0, 0);
          }
        }
        if constexpr (UB == 1) {
          if (has_next) rd(bn, t);
        }
      }
      // (Waves 4-7 filtering the previous tile before multiplying this one, so each SIMD
      // overlaps one wave's MFMAs with its partner's filter, measured slower: scan 2.51-2.55
      // against 2.19 ms at top-10.)
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) filt(acc[ub], ub, bs[bc][i], t0);
      if (t0 + 2 * kItemTile < it1) {
        put(bn2);
        if (t0 + 3 * kItemTile < it1) fetch(t0 + 3 * kItemTile);
      }
      __syncthreads();
      bc = bn;
    }
  }
  if (staged)
    flush_grouped<NU>(staged, slot0, user_list, count, cap, cand, wl, wi, wu, wr,
                      wp, ucnt, uoff, ubase);
}

// ---- 4. per-user selection: bitonic sort (descending) of 64-bit keys (logit key | ~item)
constexpr int kSelectMax = 8192;

// in-LDS bitonic sort of n2 (a power of two) keys, descending; the whole block participates
__device__ __forceinline__ void bitonic_desc(unsigned long long* keys, int n2) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int j = threadIdx.x; j < n2; j += blockDim.x) {
        const int p = j ^ stride;
        if (p > j) {
          const bool desc = (j & size) == 0;
          const unsigned long long x = keys[j], y = keys[p];
          if ((x < y) == desc) { keys[j] = y; keys[p] = x; }
        }
      }
      __syncthreads();
    }
  }
}

// Per user: the K best candidates without sorting the whole list.  The candidates' order keys
// (fkey of the logit) go to LDS; a radix select over key - min (8-bit digits from the highest bit
// the keys differ in; the wave-scan digit walk of the threshold kernel) finds the K-th largest key
// t; candidates above t, and the needed number of those equal to t (the smallest item ids: a
// second radix select over ~id, only when the tie is split), are gathered and only those K are
// sorted (bitonic over next_pow2(K) keys (logit key << 32 | ~id), descending).
// RS (rescore, the two-term split scan's candidates): the scan's logits are within E =
// c |q_u| max|p| of fp32, so the exact top K lie among the candidates whose scan logit is >=
// (the scan's K-th largest) - 2E; only those are re-scored in fp32 (logit = bias + sum_k q_k p_k,
// fmaf in k order) and the select runs on the re-scored keys (the others keyed 0: below every
// real logit's key).
// ---- 2'. the threshold sample on bf16 matrix cores (k_sample16, ncf_score_sample_split16):
// logits of n users x S sample items (sample item j = item j * stride of the index) from the
// two-term operand split (a0 b0 + a0 b1 + a1 b0 on v_mfma_f32_32x32x16_bf16: within E_u = 1e-4
// |q_u| max|p| of the fp32 logit, the scan's own two-term bound), plus the sample bias, stored
// as fp16 rounded toward -inf.  A stored value is then <= the approximate logit, so the K-th
// largest stored value v has K sample items with fp32 logit >= v - E_u: the caller lowers the
// k-th threshold by E_u (ncf_score_margin) and it stays a valid lower bound of the K-th largest.
// Against the fp32 sample GEMM: 16x the matrix rate, half the bytes written and re-read (fp16).
// Workgroup: 128 sample items staged in LDS (both planes), 4 waves x 32 users, each wave four
// 32 x 32 tiles (one per 32 items).
// G > 1: only the maximum of each group of G consecutive sample items is stored (out row length
// Sg = ceil(S / G)), reduced across the G lanes that hold the group before the one rounding
// (round-down is monotone: the stored value is the group's largest stored G = 1 value, bit for
// bit).  The K-th largest group maximum v has K distinct items at or above it, so it is <= the
// K-th largest of the whole sample and the same bound argument holds; the sample's write and
// the k-th select's read shrink G times.
template <int T, int G>
__global__ __launch_bounds__(256) void k_sample16(const float* __restrict__ q, int64_t n_users,
                                                  const uint16_t* __restrict__ items3,
                                                  int64_t n_items, int64_t stride,
                                                  const float* __restrict__ sbias, int64_t S,
                                                  _Float16* __restrict__ out) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16 || G == 32, "group of lanes");
  const int64_t Sg = (S + G - 1) / G;
  constexpr int D = 64, J = 128;
  __shared__ __attribute__((aligned(16))) uint16_t ps[T][J][kP3];
  __shared__ float bs[J];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 31, h = lane >> 5;
  const int64_t j0 = (int64_t)blockIdx.x * J;
  const int64_t u0 = (int64_t)blockIdx.y * 128 + 32 * w;
  // the sample rows' loads, then this lane's query split (the rows land meanwhile)
  constexpr int CH = T * J * (D / 8);   // 16-B chunks
  uint4 pv[CH / 256];
#pragma unroll
  for (int c = 0; c < CH / 256; ++c) {
    const int e = tid + 256 * c, pl = e / (J * 8), jj = (e / 8) % J, k8 = (e % 8) * 8;
    const int64_t j = j0 + jj;
    pv[c] = j < S ? *reinterpret_cast<const uint4*>(items3 + (int64_t)pl * n_items * D + j * stride * D + k8)
                  : make_uint4(0u, 0u, 0u, 0u);
  }
  const float bb0 = tid < J && j0 + tid < S ? sbias[j0 + tid] : 0.0f;
  bf16x8_t a[T][4];
  {
    const int64_t u = u0 + i < n_users ? u0 + i : n_users - 1;
    const float* qp = q + u * D + 32 * h;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 x = ld4(qp + 8 * t), y = ld4(qp + 8 * t + 4);
      const float v[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
      for (int jv = 0; jv < 8; ++jv) {
        __bf16 b0, b1, b2;
        split3(v[jv], b0, b1, b2);
        a[0][t][jv] = b0;
        if (T > 1) a[T > 1 ? 1 : 0][t][jv] = b1;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CH / 256; ++c) {
    const int e = tid + 256 * c, pl = e / (J * 8), jj = (e / 8) % J, k8 = (e % 8) * 8;
    *reinterpret_cast<uint4*>(&ps[pl][jj][k8]) = pv[c];
  }
  if (tid < J) bs[tid] = bb0;
  __syncthreads();
#pragma unroll
  for (int jt = 0; jt < J / 32; ++jt) {
    f32x16 acc = {};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8_t b0 = *reinterpret_cast<const bf16x8_t*>(&ps[0][32 * jt + i][32 * h + 8 * t]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][t], b0, acc, 0, 0, 0);
      if (T > 1) {
        const bf16x8_t b1 = *reinterpret_cast<const bf16x8_t*>(&ps[T > 1 ? 1 : 0][32 * jt + i][32 * h + 8 * t]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][t], b1, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[T > 1 ? 1 : 0][t], b0, acc, 0, 0, 0);
      }
    }
    const int64_t j = j0 + 32 * jt + i;
    if constexpr (G == 1) {
      if (j < S) {
        const float b = bs[32 * jt + i];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t u = u0 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (u < n_users)
            out[u * S + j] = __builtin_bit_cast(_Float16, __ocml_cvtrtn_f16_f32(acc[r] + b));
        }
      }
    } else {   // (j0 and the 32-item tiles are multiples of G: a group never spans two tiles)
      const float b = bs[32 * jt + i];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = j < S ? acc[r] + b : -INFINITY;
#pragma unroll
        for (int o = 1; o < G; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
        const int64_t u = u0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (i % G == 0 && j < S && u < n_users)
          out[u * Sg + j / G] = __builtin_bit_cast(_Float16, __ocml_cvtrtn_f16_f32(v));
      }
    }
  }
}

// The group-maxima form of k_sample16 (G = 8) with the MFMA operands swapped: items are the A
// operand (rows of the accumulator) and users the B operand (its columns), and the 32 items of a
// tile are laid along the rows so that the eight accumulator registers a lane holds for rows
// {0-3, 8-11} + 4h (and {16-19, 24-27} + 4h) are eight consecutive sample items: a group's
// maximum is a register max, no cross-lane shuffles.  The lane's group maxima go to LDS and
// leave as whole 32-byte runs of each user's row (16 groups per workgroup), instead of 2-byte
// stores scattered over 32 rows.  Users vary fastest over the grid, so the ~80 workgroups that
// read one 128-item block of the sample run back to back (one fetch per XCD, not one per user
// block).  The same products in the same order per element (p0 q0, p1 q0, p0 q1 against k_sample16's
// q0 p0, q0 p1, q1 p0), the same rounding: bit for bit k_sample16<T, 8>.
template <int T>
__global__ __launch_bounds__(256) void k_sample16t(const float* __restrict__ q, int64_t n_users,
                                                   const uint16_t* __restrict__ items3,
                                                   int64_t n_items, int64_t stride,
                                                   const float* __restrict__ sbias, int64_t S,
                                                   _Float16* __restrict__ out) {
  constexpr int D = 64, J = 128, G = 8, NG = J / G;
  const int64_t Sg = (S + G - 1) / G;
  __shared__ __attribute__((aligned(16))) uint16_t ps[T][J][kP3];
  __shared__ float bs[J];
  __shared__ _Float16 og[4][32][NG + 2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 31, h = lane >> 5;
  const int64_t u0 = (int64_t)blockIdx.x * 128 + 32 * w;
  const int64_t j0 = (int64_t)blockIdx.y * J;
  constexpr int CH = T * J * (D / 8);   // 16-B chunks
  uint4 pv[CH / 256];
#pragma unroll
  for (int c = 0; c < CH / 256; ++c) {
    const int e = tid + 256 * c, pl = e / (J * 8), jj = (e / 8) % J, k8 = (e % 8) * 8;
    const int64_t j = j0 + jj;
    pv[c] = j < S ? *reinterpret_cast<const uint4*>(items3 + (int64_t)pl * n_items * D + j * stride * D + k8)
                  : make_uint4(0u, 0u, 0u, 0u);
  }
  const float bb0 = tid < J && j0 + tid < S ? sbias[j0 + tid] : 0.0f;
  bf16x8_t b[T][4];   // this lane's user (column i), k = 32 h + 8 t .. + 7 of chunk t
  {
    const int64_t u = u0 + i < n_users ? u0 + i : n_users - 1;
    const float* qp = q + u * D + 32 * h;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 x = ld4(qp + 8 * t), y = ld4(qp + 8 * t + 4);
      const float v[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
      for (int jv = 0; jv < 8; ++jv) {
        __bf16 b0, b1, b2;
        split3(v[jv], b0, b1, b2);
        b[0][t][jv] = b0;
        if (T > 1) b[T > 1 ? 1 : 0][t][jv] = b1;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CH / 256; ++c) {
    const int e = tid + 256 * c, pl = e / (J * 8), jj = (e / 8) % J, k8 = (e % 8) * 8;
    *reinterpret_cast<uint4*>(&ps[pl][jj][k8]) = pv[c];
  }
  if (tid < J) bs[tid] = j0 + tid < S ? bb0 : -INFINITY;   // (past S: the group max's -inf)
  __syncthreads();
  // accumulator row m = (r & 3) + 8 (r >> 2) + 4 h holds tile item it(m): rows of register
  // quarter q = r >> 2 and half h -> group 2 (q >> 1) + h, position (r & 3) + 4 (q & 1)
  const int mrow = i;   // this lane's A row
  const int it_a = 8 * (2 * ((mrow >> 3) >> 1) + ((mrow >> 2) & 1)) + (mrow & 3) + 4 * ((mrow >> 3) & 1);
#pragma unroll
  for (int jt = 0; jt < J / 32; ++jt) {
    f32x16 acc = {};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(&ps[0][32 * jt + it_a][32 * h + 8 * t]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[0][t], acc, 0, 0, 0);
      if (T > 1) {
        const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(&ps[T > 1 ? 1 : 0][32 * jt + it_a][32 * h + 8 * t]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[0][t], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[T > 1 ? 1 : 0][t], acc, 0, 0, 0);
      }
    }
    float g[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const float* bg = bs + 32 * jt + 8 * (2 * half + h);   // the group's 8 biases (broadcast)
      float v = -INFINITY;
#pragma unroll
      for (int r = 8 * half; r < 8 * half + 8; ++r)
        v = fmaxf(v, acc[r] + bg[(r & 3) + 4 * ((r >> 2) & 1)]);
      g[half] = v;
    }
    og[w][i][4 * jt + h] = __builtin_bit_cast(_Float16, __ocml_cvtrtn_f16_f32(g[0]));
    og[w][i][4 * jt + 2 + h] = __builtin_bit_cast(_Float16, __ocml_cvtrtn_f16_f32(g[1]));
  }
  __syncthreads();
  // the wave's 32 users x 16 groups: 16 consecutive lanes write one user's 32-byte run
  const int64_t g0 = j0 / G;
#pragma unroll
  for (int s = 0; s < 32 * NG / 64; ++s) {
    const int e = lane + 64 * s, uu = e / NG, gl = e % NG;
    const int64_t u = u0 + uu;
    if (u < n_users && g0 + gl < Sg) out[u * Sg + g0 + gl] = og[w][uu][gl];
  }
}

template <bool RS>
__global__ __launch_bounds__(256) void k_select(const int32_t* __restrict__ user_list,
                                                int64_t n_users, const uint32_t* __restrict__ count,
                                                const ncf_score_cand* __restrict__ cand,
                                                int64_t cap, int K, int n2K,
                                                const float* __restrict__ q,
                                                const float* __restrict__ items,
                                                const float* __restrict__ item_bias,
                                                const uint32_t* __restrict__ pmax, float c,
                                                float* __restrict__ out_score,
                                                int64_t* __restrict__ out_item,
                                                float* __restrict__ thr_out,
                                                uint32_t* __restrict__ overflow,
                                                const float* __restrict__ thr_check) {
  extern __shared__ unsigned long long sel[];   // [n2K] selected keys, then uint32 keys[cap]
  uint32_t* keys = reinterpret_cast<uint32_t*>(sel + n2K);
  __shared__ uint32_t hist[256];
  __shared__ uint32_t rmin[4], rmax[4], rcnt[4];
  __shared__ uint32_t s_dig, s_need, s_eq, s_n;
  const int64_t slot = blockIdx.x;
  if (slot >= n_users) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t u = user_list ? user_list[slot] : slot;
  const uint32_t c_all = count[u];
  const int nc = (int)(c_all < cap ? c_all : cap);
  const ncf_score_cand* cc = cand + u * cap;   // (logit, item) records
  // block min / max of the keys of the members (key != 0) and their number
  auto key_range = [&](uint32_t& kmin, uint32_t& kmax, uint32_t& nmem) {
    kmin = 0xFFFFFFFFu; kmax = 0; nmem = 0;
    for (int j = tid; j < nc; j += 256) {
      const uint32_t k = keys[j];
      if (k == 0) continue;
      kmin = min(kmin, k);
      kmax = max(kmax, k);
      ++nmem;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o, 64));
      kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
      nmem += (uint32_t)__shfl_xor((int)nmem, o, 64);
    }
    if (lane == 0) { rmin[w] = kmin; rmax[w] = kmax; rcnt[w] = nmem; }
    __syncthreads();
    kmin = min(min(rmin[0], rmin[1]), min(rmin[2], rmin[3]));
    kmax = max(max(rmax[0], rmax[1]), max(rmax[2], rmax[3]));
    nmem = (rcnt[0] + rcnt[1]) + (rcnt[2] + rcnt[3]);
    __syncthreads();
  };
  // radix select of one key domain: the need-th largest value among the members; returns the
  // value, *need_left = members equal to it still needed, *n_eq = members equal to it
  auto radix = [&](auto member, auto value, int nbits, uint32_t need, uint32_t* need_left,
                   uint32_t* n_eq) -> uint32_t {
    uint32_t prefix = 0, eq = 0;
    for (int hi = nbits; hi > 0;) {
      const int lo = hi > 8 ? hi - 8 : 0;
      const uint32_t dm = (1u << (hi - lo)) - 1u;
      hist[tid] = 0;
      __syncthreads();
      for (int j = tid; j < nc; j += 256) {
        if (!member(j)) continue;
        const uint32_t d = value(j);
        if (hi >= 32 || (d >> hi) == (prefix >> hi)) atomicAdd(&hist[(d >> lo) & dm], 1u);
      }
      __syncthreads();
      if (w == 0) {
        uint32_t above = 0;
        const int dig = kth_walk(hist, need, &above);
        if (lane == 0) { s_dig = (uint32_t)dig; s_need = need - above; s_eq = hist[dig]; }
      }
      __syncthreads();
      prefix |= s_dig << lo;
      need = s_need;
      eq = s_eq;
      hi = lo;
      __syncthreads();
    }
    *need_left = need;
    *n_eq = eq;
    return prefix;
  };
  // the key of the K-th largest member (span 0: every member equal)
  auto kth_key = [&](uint32_t kmin, uint32_t kmax, uint32_t nmem, uint32_t* need,
                     uint32_t* eq) -> uint32_t {
    const uint32_t span = kmax - kmin;
    const int nb = span ? 32 - __builtin_clz(span) : 0;
    *need = (uint32_t)K;
    *eq = nmem;
    if (nb == 0) return kmin;
    return kmin + radix([&](int j) { return keys[j] != 0; }, [&](int j) { return keys[j] - kmin; },
                        nb, (uint32_t)K, need, eq);
  };
  if (tid == 0) s_n = 0;
  for (int j = tid; j < nc; j += 256) keys[j] = fkey(cc[j].logit);
  __syncthreads();
  uint32_t kmin, kmax, nmem;
  key_range(kmin, kmax, nmem);
  if constexpr (RS) {
    float qr[64];
    float qq = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; k += 4) {
      const float4 x = ld4(q + u * 64 + k);
      qr[k] = x.x; qr[k + 1] = x.y; qr[k + 2] = x.z; qr[k + 3] = x.w;
      qq += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    }
    float lo = -INFINITY;   // re-score the candidates with a scan logit >= lo
    if (nmem > (uint32_t)K) {
      uint32_t need, eq;
      const float va = fkey_inv(kth_key(kmin, kmax, nmem, &need, &eq));
      const float e = c * sqrtf(qq) * __uint_as_float(*pmax);
      lo = va - (2.0f * e * 1.0001f + 1e-6f * fabsf(va));
    }
    for (int j = tid; j < nc; j += 256) {
      const ncf_score_cand rc = cc[j];
      if (rc.logit < lo) { keys[j] = 0; continue; }
      const int64_t it = rc.item;
      const float* pr = items + it * 64;
      float d = 0.0f;
#pragma unroll
      for (int k = 0; k < 64; k += 4) {
        const float4 x = ld4(pr + k);
        d = fmaf(qr[k], x.x, d);
        d = fmaf(qr[k + 1], x.y, d);
        d = fmaf(qr[k + 2], x.z, d);
        d = fmaf(qr[k + 3], x.w, d);
      }
      keys[j] = fkey(d + item_bias[it]);
    }
    __syncthreads();
    key_range(kmin, kmax, nmem);
  }
  const int ne = (int)nmem;     // members (RS: the re-scored candidates)
  uint32_t t = 0, t2 = 0;       // take key > t; key == t: all (tie_all) or ~id >= t2
  bool tie_all = true;
  if (ne > K) {
    uint32_t need = (uint32_t)K, eq = nmem;
    t = kth_key(kmin, kmax, nmem, &need, &eq);
    if (eq > need) {   // the tie at t is split: the smallest ids among the keys equal to t
      tie_all = false;
      uint32_t need2 = 0, eq2 = 0;
      t2 = radix([&](int j) { return keys[j] == t; },
                 [&](int j) { return 0xFFFFFFFFu - (uint32_t)cc[j].item; }, 32, need, &need2, &eq2);
    }
  }
  for (int j = tid; j < nc; j += 256) {
    const uint32_t k = keys[j];
    if (k == 0) continue;
    if (ne > K && k < t) continue;
    const uint32_t nid = 0xFFFFFFFFu - (uint32_t)cc[j].item;
    if (ne > K && k == t && !tie_all && nid < t2) continue;
    const uint32_t pos = atomicAdd(&s_n, 1u);   // (exactly min(ne, K) arrive)
    if (pos < (uint32_t)n2K) sel[pos] = ((unsigned long long)k << 32) | (unsigned long long)nid;
  }
  __syncthreads();
  const int ns = min((int)s_n, K);   // = min(ne, K)
  for (int j = ns + tid; j < n2K; j += 256) sel[j] = 0ull;
  __syncthreads();
  bitonic_desc(sel, n2K);
  for (int j = tid; j < K; j += 256) {
    const unsigned long long k = sel[j];
    const bool ok = j < ns;
    const float lg = fkey_inv((uint32_t)(k >> 32));
    out_score[slot * K + j] = ok ? 1.0f / (1.0f + expf(-lg)) : 0.0f;
    out_item[slot * K + j] = ok ? (int64_t)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)) : -1;
  }
  if (tid == 0) {
    const bool over = c_all > (uint32_t)cap;
    // thr_check (a rank-j threshold, j < K: not a guaranteed bound of the K-th logit): the scan
    // collected every item whose fp32 logit is >= thr_check[u], so the K selected are the top K
    // iff K were selected and the K-th of them is >= it; else flag 2 (the host re-runs the user
    // from the sample's K-th, a guaranteed bound)
    const bool under = !over && thr_check &&
        (ns < K || fkey_inv((uint32_t)(sel[K - 1] >> 32)) < thr_check[u]);
    overflow[slot] = over ? 1u : (under ? 2u : 0u);
    // a valid higher threshold for a re-run: the K-th best of the candidates seen
    if (over && thr_out) thr_out[u] = fkey_inv((uint32_t)(sel[K - 1] >> 32));
  }
}

// ---- 5. merge of per-shard top-K lists (item-sharded scoring): per user, the L
// candidates (score, global item id; id < 0 = empty) sorted by (score desc, item id asc)
__global__ __launch_bounds__(1024) void k_merge(const float* __restrict__ cand_score,
                                                const int64_t* __restrict__ cand_item, int64_t L,
                                                int K, float* __restrict__ out_score,
                                                int64_t* __restrict__ out_item) {
  extern __shared__ unsigned long long keys[];
  const int64_t u = blockIdx.x;
  int n2 = 1;
  while (n2 < L || n2 < K) n2 <<= 1;
  for (int j = threadIdx.x; j < n2; j += blockDim.x) {
    unsigned long long k = 0ull;
    if (j < L) {
      const int64_t id = cand_item[u * L + j];
      if (id >= 0)
        k = ((unsigned long long)fkey(cand_score[u * L + j]) << 32) |
            (unsigned long long)(0xFFFFFFFFu - (uint32_t)id);
    }
    keys[j] = k;
  }
  __syncthreads();
  bitonic_desc(keys, n2);
  for (int j = threadIdx.x; j < K; j += blockDim.x) {
    const unsigned long long k = keys[j];
    const bool ok = k != 0ull;
    out_score[u * K + j] = ok ? fkey_inv((uint32_t)(k >> 32)) : 0.0f;
    out_item[u * K + j] = ok ? (int64_t)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)) : -1;
  }
}

}  // namespace

extern "C" int ncf_score_merge(const float* cand_score, const int64_t* cand_item, int64_t n_users,
                               int64_t L, int K, float* out_score, int64_t* out_item,
                               void* stream) {
  NCF_CHECK_ARG(n_users >= 0 && K >= 1 && L >= 1 && L <= kSelectMax && K <= kSelectMax,
                "ncf_score_merge: need 1 <= K, L <= %d", kSelectMax);
  if (n_users == 0) return NCF_OK;
  int n2 = 1;
  while (n2 < L || n2 < K) n2 <<= 1;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_merge, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(sizeof(unsigned long long) * kSelectMax));
    attr = true;
  }
  hipLaunchKernelGGL(k_merge, dim3((unsigned)n_users), dim3(1024),
                     sizeof(unsigned long long) * (size_t)n2, (hipStream_t)stream, cand_score,
                     cand_item, L, K, out_score, out_item);
  NCF_CHECK_LAUNCH("ncf_score_merge");
  return NCF_OK;
}

extern "C" int ncf_score_queries(const int64_t* user_ids, int64_t n, const float* mf_user,
                                 int64_t rows, int64_t dim, const float* mf_gamma,
                                 const float* mf_beta, float eps, const float* mf_out_w,
                                 const float* final_w, float* queries, int* err_flag,
                                 void* stream) {
  NCF_CHECK_ARG(n >= 0 && (dim == 16 || dim == 32 || dim == 64 || dim == 128),
                "ncf_score_queries: dim must be 16, 32, 64 or 128");
  if (n == 0) return NCF_OK;
#define NCF_QUERIES(DD)                                                                           \
  if (dim == DD)                                                                                  \
    hipLaunchKernelGGL(k_queries<DD>, dim3(ncf_cdiv(n * (DD / 4), 256)), dim3(256), 0,            \
                       (hipStream_t)stream, user_ids, n, mf_user, rows, mf_gamma, mf_beta, eps,     \
                       mf_out_w, final_w, queries, err_flag);
  NCF_QUERIES(16) NCF_QUERIES(32) NCF_QUERIES(64) NCF_QUERIES(128)
#undef NCF_QUERIES
  NCF_CHECK_LAUNCH("ncf_score_queries");
  return NCF_OK;
}

extern "C" int ncf_score_item_bias(const float* mlp_item, int64_t n, const float* final_w,
                                   const float* final_b, const float* mf_out_b, float* bias,
                                   void* stream) {
  NCF_CHECK_ARG(n >= 0, "ncf_score_item_bias: n < 0");
  if (n == 0) return NCF_OK;
  hipLaunchKernelGGL(k_item_bias, dim3(ncf_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     mlp_item, n, final_w, final_b, mf_out_b, bias);
  NCF_CHECK_LAUNCH("ncf_score_item_bias");
  return NCF_OK;
}

extern "C" int ncf_score_kth(const float* logits, int64_t n_users, int64_t S, int K,
                             const float* item_bias, int64_t stride, float* thr, void* stream) {
  NCF_CHECK_ARG(n_users >= 0 && S >= 1 && K >= 1 && stride >= 1, "ncf_score_kth: bad size");
  if (n_users == 0) return NCF_OK;
  // The LDS-resident sample needs 4 S bytes of dynamic LDS (152 KB at kKthLdsMax: a 160 KB
  // part).  The limit is taken from the device once: a part with less LDS, or an attribute the
  // runtime refuses, sends every sample to the streaming k_kth instead of failing the launch.
  static int64_t lds_max = -1;
  if (lds_max < 0) {
    int dev = 0, smem = 0;
    int64_t lim = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&smem, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess) {
      lim = ((int64_t)smem - 8192) / (int64_t)sizeof(uint32_t);   // static LDS of k_kth_lds < 8 KB
      lim = lim < kKthLdsMax ? lim : kKthLdsMax;
    }
    const int bytes = (int)(sizeof(uint32_t) * (lim > 0 ? lim : 1));
    if (lim <= 0 ||
        hipFuncSetAttribute((const void*)k_kth_lds<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            bytes) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_kth_lds<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            bytes) != hipSuccess) {
      (void)hipGetLastError();
      lim = 0;
    }
    lds_max = lim;
  }
  if (S <= lds_max) {
    // measured: S = 38912 (top-100) 0.75 -> 0.55 ms with 1024 threads; S = 9984 (top-10) 0.12 ms
    // with 512 against 0.16 with 1024
    if (S > 16384)
      hipLaunchKernelGGL(k_kth_lds<1024>, dim3((unsigned)n_users), dim3(1024),
                         sizeof(uint32_t) * S, (hipStream_t)stream, logits, S, K, item_bias, stride,
                         thr);
    else
      hipLaunchKernelGGL(k_kth_lds<512>, dim3((unsigned)n_users), dim3(512), sizeof(uint32_t) * S,
                         (hipStream_t)stream, logits, S, K, item_bias, stride, thr);
  } else {
    hipLaunchKernelGGL(k_kth, dim3((unsigned)n_users), dim3(256), 0, (hipStream_t)stream, logits,
                       S, K, item_bias, stride, thr);
  }
  NCF_CHECK_LAUNCH("ncf_score_kth");
  return NCF_OK;
}

// The fp16 threshold sample of k_sample16 (bias included, rounded down) and its k-th (LDS-
// resident fp16 rows: S <= kKthLdsMax).
extern "C" int ncf_score_sample_split16(const float* queries, int64_t n_users,
                                        const uint16_t* items3, int64_t n_items, int64_t dim,
                                        int64_t stride, const float* sample_bias, int64_t S,
                                        int64_t group, uint16_t* out, void* stream) {
  NCF_CHECK_ARG(dim == 64, "ncf_score_sample_split16: dim must be 64");
  NCF_CHECK_ARG(n_users >= 0 && S >= 1 && stride >= 1 && (S - 1) * stride < n_items &&
                    (group == 1 || group == 8) && queries && items3 && sample_bias && out,
                "ncf_score_sample_split16: bad args");
  if (n_users == 0) return NCF_OK;
  const dim3 grid((unsigned)ncf_cdiv(S, 128), (unsigned)ncf_cdiv(n_users, 128));
  _Float16* o = reinterpret_cast<_Float16*>(out);
  if (group == 8) {
    NCF_CHECK_ARG(ncf_cdiv(S, 128) <= 65535, "ncf_score_sample_split16: S too large");
    const dim3 gt((unsigned)ncf_cdiv(n_users, 128), (unsigned)ncf_cdiv(S, 128));
    hipLaunchKernelGGL((k_sample16t<2>), gt, dim3(256), 0, (hipStream_t)stream, queries,
                       n_users, items3, n_items, stride, sample_bias, S, o);
  } else
    hipLaunchKernelGGL((k_sample16<2, 1>), grid, dim3(256), 0, (hipStream_t)stream, queries,
                       n_users, items3, n_items, stride, sample_bias, S, o);
  NCF_CHECK_LAUNCH("ncf_score_sample_split16");
  return NCF_OK;
}

extern "C" int ncf_score_kth16(const uint16_t* logits, int64_t n_users, int64_t S, int K,
                               float* thr, void* stream) {
  NCF_CHECK_ARG(n_users >= 0 && S >= 1 && S <= kKthLdsMax && K >= 1 && logits && thr,
                "ncf_score_kth16: bad size");
  if (n_users == 0) return NCF_OK;
  static bool attr = false;
  if (!attr) {
    const int bytes = (int)(sizeof(_Float16) * kKthLdsMax);
    if (hipFuncSetAttribute((const void*)k_kth_lds<512, _Float16>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_kth_lds<1024, _Float16>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
      ncf_set_error("ncf_score_kth16: %d B of LDS refused", bytes);
      return NCF_ERR_LAUNCH;
    }
    attr = true;
  }
  const _Float16* l = reinterpret_cast<const _Float16*>(logits);
  if (S > 16384)
    hipLaunchKernelGGL((k_kth_lds<1024, _Float16>), dim3((unsigned)n_users), dim3(1024),
                       sizeof(_Float16) * S, (hipStream_t)stream, l, S, K, nullptr, 1, thr);
  else
    hipLaunchKernelGGL((k_kth_lds<512, _Float16>), dim3((unsigned)n_users), dim3(512),
                       sizeof(_Float16) * S, (hipStream_t)stream, l, S, K, nullptr, 1, thr);
  NCF_CHECK_LAUNCH("ncf_score_kth16");
  return NCF_OK;
}

extern "C" int ncf_score_collect(const float* queries, const int32_t* user_list, int64_t n_users,
                                 const float* items, const float* item_bias, int64_t n_items,
                                 int64_t dim, const float* thr, int64_t cap, uint32_t* count,
                                 ncf_score_cand* cand, void* stream) {
  NCF_CHECK_ARG(dim == 64 || dim == 128, "ncf_score_collect: dim must be 64 or 128");
  NCF_CHECK_ARG(n_users >= 0 && n_items >= 0 && n_items < (1ll << 31) && cap >= 1,
                "ncf_score_collect: bad size");
  if (n_users == 0 || n_items == 0) return NCF_OK;
  // item split: enough workgroups to fill the chip (>= ~2 per CU) with >= 8 tiles each
  const int64_t ub = (n_users + kUsersPerBlock - 1) / kUsersPerBlock;
  int64_t splits = (1024 + ub - 1) / ub;
  const int64_t max_splits = (n_items + 8 * kItemTile - 1) / (8 * kItemTile);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int64_t per = (n_items + splits - 1) / splits;
  per = (per + kItemTile - 1) / kItemTile * kItemTile;
  splits = (n_items + per - 1) / per;
  NCF_CHECK_ARG(ub < 65536, "ncf_score_collect: too many users per call (max %d)", 65535 * 256);
  if (dim == 64)
    hipLaunchKernelGGL(k_collect<64>, dim3((unsigned)splits, (unsigned)ub), dim3(512), 0,
                       (hipStream_t)stream, queries, user_list, n_users, items, item_bias, n_items,
                       per, thr, cap, count, cand);
  else
    hipLaunchKernelGGL(k_collect<128>, dim3((unsigned)splits, (unsigned)ub), dim3(512), 0,
                       (hipStream_t)stream, queries, user_list, n_users, items, item_bias, n_items,
                       per, thr, cap, count, cand);
  NCF_CHECK_LAUNCH("ncf_score_collect");
  return NCF_OK;
}

// three bf16 planes [3][n_items][dim] of the item rows (the operand split of
// ncf_score_collect_split; built once per item index)
extern "C" int ncf_score_split_items(const float* items, int64_t n_items, int64_t dim,
                                     uint16_t* items3, void* stream) {
  NCF_CHECK_ARG(n_items >= 0 && dim >= 1 && items && items3, "ncf_score_split_items: bad args");
  const int64_t n = n_items * dim;
  if (n == 0) return NCF_OK;
  hipLaunchKernelGGL(k_split3, dim3((unsigned)ncf_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     items, n, items3);
  NCF_CHECK_LAUNCH("ncf_score_split_items");
  return NCF_OK;
}

extern "C" int ncf_score_item_norm_max(const float* items, int64_t n_items, int64_t dim,
                                       uint32_t* out_bits, void* stream) {
  NCF_CHECK_ARG(dim == 64 && n_items >= 0 && out_bits, "ncf_score_item_norm_max: dim must be 64");
  (void)hipMemsetAsync(out_bits, 0, sizeof(uint32_t), (hipStream_t)stream);
  if (n_items == 0) return NCF_OK;
  NCF_CHECK_ARG(((uintptr_t)items & 15) == 0, "ncf_score_item_norm_max: rows must be 16-B aligned");
  const int64_t blocks = std::min<int64_t>(kNormMaxBlocks, ncf_cdiv(n_items, 16));
  hipLaunchKernelGGL(k_row_norm_max, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, items, n_items, out_bits);
  NCF_CHECK_LAUNCH("ncf_score_item_norm_max");
  return NCF_OK;
}

extern "C" int ncf_score_margin(const float* queries, const int32_t* user_list, int64_t n_users,
                                int64_t dim, const uint32_t* item_norm_max, float c, float* thr,
                                void* stream) {
  NCF_CHECK_ARG(dim == 64 && n_users >= 0 && c >= 0.0f, "ncf_score_margin: dim must be 64");
  if (n_users == 0) return NCF_OK;
  hipLaunchKernelGGL(k_score_margin, dim3((unsigned)ncf_cdiv(n_users, 4)), dim3(256), 0,
                     (hipStream_t)stream, queries, user_list, n_users, item_norm_max, c, thr);
  NCF_CHECK_LAUNCH("ncf_score_margin");
  return NCF_OK;
}

// ncf_score_collect on bf16 matrix cores with fp32 accuracy (three-term operand split, six
// products; items3 from ncf_score_split_items): the same candidate sets
extern "C" int ncf_score_collect_split(const float* queries, const int32_t* user_list,
                                       int64_t n_users, const uint16_t* items3,
                                       const float* item_bias, int64_t n_items, int64_t dim,
                                       const float* thr, int64_t cap, uint32_t* count,
                                       ncf_score_cand* cand, int terms,
                                       int64_t expected_per_user, void* stream) {
  NCF_CHECK_ARG(terms >= 1 && terms <= 3, "ncf_score_collect_split: terms must be 1, 2 or 3");
  NCF_CHECK_ARG(dim == 64, "ncf_score_collect_split: dim must be 64");
  NCF_CHECK_ARG(n_users >= 0 && n_items >= 0 && n_items < (1ll << 31) && cap >= 1,
                "ncf_score_collect_split: bad size");
  if (n_users == 0 || n_items == 0) return NCF_OK;
  // Grid: (item split x user block) workgroups (one per CU: 8 waves at two per SIMD), sized in
  // whole rounds of the chip's CUs — every workgroup scans the same number of tiles, so a partial
  // last round would cost a whole round.  At least ~4 rounds, >= 8 tiles per workgroup.
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n_cu = v;
    else
      n_cu = 256;
  }
  const int nub = terms == 3 ? kUB3t : kUB3;
  const int64_t upb = 32 * kNW3 * nub;   // users per workgroup
  const int64_t ub = (n_users + upb - 1) / upb;
  NCF_CHECK_ARG(ub < (1ll << 24), "ncf_score_collect_split: too many users per call");
  const int64_t max_splits = std::max<int64_t>(1, (n_items + 8 * kItemTile - 1) / (8 * kItemTile));
  const int64_t slots = (int64_t)n_cu * (8 / kNW3);   // resident workgroups (2 waves/SIMD)
  const int min_rounds = 4;    // at least this many rounds of resident workgroups
  int64_t splits = (min_rounds * slots + ub - 1) / ub;
  if (expected_per_user > 0) {
    // enough item splits that a wave's share of its users' candidates (expected x 32 UB users /
    // splits) stays under 3/4 of its LDS slice: a slice that fills inside the scan loop is
    // written out one candidate at a time (k_collect3).  PMC writes per scan (MB), top-10 /
    // top-100: 64 splits 329 / 1175, 128 splits 219 / 1045, 256 splits 298 / 622; scan time
    // unchanged
    const int64_t slice = terms == 3 ? slice3<3>() : terms == 2 ? slice3<2>() : slice3<1>();
    const int64_t need = (expected_per_user * 32 * nub * 4 + 3 * slice - 1) / (3 * slice);
    splits = std::max(splits, need);
  }
  const int64_t rounds = (splits * ub + slots - 1) / slots;
  splits = std::max<int64_t>(1, rounds * slots / ub);
  if (splits > max_splits) splits = max_splits;
  int64_t per = (n_items + splits - 1) / splits;
  per = (per + kItemTile - 1) / kItemTile * kItemTile;
  splits = (n_items + per - 1) / per;
  NCF_CHECK_ARG(splits * ub < (1ll << 31), "ncf_score_collect_split: grid too large");
  const size_t dyn = (size_t)kNW3 * (terms == 3   ? slice3_bytes<kUB3t, 3>()
                                     : terms == 2 ? slice3_bytes<kUB3, 2>()
                                                  : slice3_bytes<kUB3, 1>());
  static bool attr3 = false;
  if (!attr3) {
    const hipError_t e0 = hipFuncSetAttribute((const void*)k_collect3<kUB3t, kNW3, 3>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)(kNW3 * slice3_bytes<kUB3t, 3>()));
    const hipError_t e1 = hipFuncSetAttribute((const void*)k_collect3<kUB3, kNW3, 2>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)(kNW3 * slice3_bytes<kUB3, 2>()));
    const hipError_t e2 = hipFuncSetAttribute((const void*)k_collect3<kUB3, kNW3, 1, kScanNB>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)(kNW3 * slice3_bytes<kUB3, 1>()));
    if (e0 != hipSuccess || e1 != hipSuccess || e2 != hipSuccess) {
      ncf_set_error("ncf_score_collect_split: candidate slices need more LDS than allowed");
      return NCF_ERR_LAUNCH;
    }
    attr3 = true;
  }
  if (terms == 3)
    hipLaunchKernelGGL((k_collect3<kUB3t, kNW3, 3>), dim3((unsigned)(splits * ub)),
                       dim3(64 * kNW3), dyn, (hipStream_t)stream, queries, user_list, n_users,
                       items3, item_bias, n_items, per, (int)ub, thr, cap, count, cand);
  else if (terms == 2)
    hipLaunchKernelGGL((k_collect3<kUB3, kNW3, 2>), dim3((unsigned)(splits * ub)),
                       dim3(64 * kNW3), dyn, (hipStream_t)stream, queries, user_list, n_users,
                       items3, item_bias, n_items, per, (int)ub, thr, cap, count, cand);
  else
    hipLaunchKernelGGL((k_collect3<kUB3, kNW3, 1, kScanNB>), dim3((unsigned)(splits * ub)),
                       dim3(64 * kNW3), dyn, (hipStream_t)stream, queries, user_list, n_users,
                       items3, item_bias, n_items, per, (int)ub, thr, cap, count, cand);
  NCF_CHECK_LAUNCH("ncf_score_collect_split");
  return NCF_OK;
}

extern "C" int ncf_score_select(const int32_t* user_list, int64_t n_users, const uint32_t* count,
                                const ncf_score_cand* cand, int64_t cap,
                                int K, float* out_score, int64_t* out_item, float* thr,
                                uint32_t* overflow, void* stream) {
  NCF_CHECK_ARG(n_users >= 0 && K >= 1 && cap >= K && cap <= kSelectMax,
                "ncf_score_select: need 1 <= K <= cap <= %d", kSelectMax);
  if (n_users == 0) return NCF_OK;
  int n2K = 1;
  while (n2K < K) n2K <<= 1;
  const size_t lds = sizeof(unsigned long long) * (size_t)n2K + sizeof(uint32_t) * (size_t)cap;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_select<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)((sizeof(unsigned long long) + sizeof(uint32_t)) * kSelectMax));
    attr = true;
  }
  hipLaunchKernelGGL(k_select<false>, dim3((unsigned)n_users), dim3(256), lds, (hipStream_t)stream,
                     user_list, n_users, count, cand, cap, K, n2K, nullptr,
                     nullptr, nullptr, nullptr, 0.0f, out_score, out_item, thr, overflow, nullptr);
  NCF_CHECK_LAUNCH("ncf_score_select");
  return NCF_OK;
}

// ncf_score_select with every candidate's logit recomputed in fp32 from queries [.., 64] and
// items [n_items, 64] + item_bias (the two-term split scan's candidates)
extern "C" int ncf_score_select_rescored(const int32_t* user_list, int64_t n_users,
                                         const uint32_t* count, const ncf_score_cand* cand,
                                         int64_t cap, int K,
                                         const float* queries, const float* items,
                                         const float* item_bias, int64_t dim,
                                         const uint32_t* item_norm_max, float c,
                                         float* out_score, int64_t* out_item, float* thr,
                                         uint32_t* overflow, const float* thr_check,
                                         void* stream) {
  NCF_CHECK_ARG(dim == 64 && queries && items && item_bias && item_norm_max,
                "ncf_score_select_rescored: dim must be 64, rows non-null");
  NCF_CHECK_ARG(n_users >= 0 && K >= 1 && cap >= K && cap <= kSelectMax,
                "ncf_score_select_rescored: need 1 <= K <= cap <= %d", kSelectMax);
  if (n_users == 0) return NCF_OK;
  int n2K = 1;
  while (n2K < K) n2K <<= 1;
  const size_t lds = sizeof(unsigned long long) * (size_t)n2K + sizeof(uint32_t) * (size_t)cap;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_select<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)((sizeof(unsigned long long) + sizeof(uint32_t)) * kSelectMax));
    attr = true;
  }
  hipLaunchKernelGGL(k_select<true>, dim3((unsigned)n_users), dim3(256), lds, (hipStream_t)stream,
                     user_list, n_users, count, cand, cap, K, n2K, queries, items,
                     item_bias, item_norm_max, c, out_score, out_item, thr, overflow, thr_check);
  NCF_CHECK_LAUNCH("ncf_score_select_rescored");
  return NCF_OK;
}
