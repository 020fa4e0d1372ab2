// The whole attention block of AdvancedNCF in one launch per direction: Q/K/V projections, the
// per-group multi-head core and out_proj, for D = 64 (C2) or D = 128 (C4) and groups of M <= 6
// rows.
//
// Reference: MultiHeadAttention.forward (src/model/architecture.py:18-57) as AdvancedNCF.forward
// calls it (:315-326): q = LN(user_mlp rows), k = v = LN(item_mlp rows), groups of
// M = 1 + negative_samples rows, Q/K/V/out Linear(D, D), scores/sqrt(hd), softmax, dropout on
// the weights, ·V, heads merged, out_proj.  Same math and the same dropout stream as the
// unfused path (gemm_rows.hip x4 + attention.hip); only the fmaf order of the projections
// differs (the k-permuted MFMA below).
//
// Tiling: a 512-thread workgroup owns G interaction groups (G = 16 at D = 64, 8 at D = 128: the
// backward's five row buffers must fit the 160 KB of LDS) = R = G*M rows, padded with zero rows
// to NT = ceil(R/16) row tiles, so every group is whole inside it and the core never leaves LDS.
// The projections are 16x16 output tiles of v_mfma_f32_16x16x4_f32 over K = D: with CS = D/16
// column slices, wave w owns output columns [16(w%CS), +16) for the row tiles rt = w/CS (mod
// 8/CS) (D = 64: two waves per column slice, row tiles of either parity; D = 128: one wave per
// slice, every row tile), its weight fragment (D/4 floats per lane) loaded once.  k-permuted
// operands: in MFMA step s, lane group g = lane>>4 supplies k = (D/4)g + s, so each lane's A row
// slice and B weight slice are D/4 contiguous floats (ds_read_b128 / global float4 runs).  Rows
// are staged in LDS with a (D+4)-float pitch (conflict-free 16-row x 4-slice fragment reads).
//
// Forward LDS: S0 = X_u -> Q -> O, S1 = X_i -> K -> Y, S2 = V   (3 x 16NT x (D+4) floats)
// Backward LDS: S0 = dY -> dO -> dX_u, S1 = Q -> dK -> dX_i, S2 = K -> dQ, S3 = V -> dV, + dS
//
// Device code (shared by attn_block.hip and the fused attention + tower kernels of tower_fused.hip):
// everything lives in namespace ncf_attn, internal linkage per translation unit.
#pragma once
#include "ncf_common.h"

namespace ncf_attn {
namespace {

constexpr int kMaxM = 6;
constexpr int kThreads = 512;   // 8 waves

#ifndef NCF_ATTN_G64
#define NCF_ATTN_G64 16   // groups per workgroup at D = 64 (build knob; 8 measured slower: 0.337 vs 0.310 ms/step)
#endif
// Geometry per embedding width D (64: C2, 128: C4)
template <int D>
struct AG {
  static constexpr int kPitch = D + 4;
  static constexpr int kGroups = D == 64 ? NCF_ATTN_G64 : 8;   // interaction groups per workgroup
  static constexpr int CS = D / 16;                  // 16-column output slices
  static constexpr int RP = 8 / CS;                  // waves per column slice (row-tile stride)
  static constexpr int KF = D / 4;                   // k values of one lane's MFMA fragment
  static constexpr int NTmax = (kGroups * kMaxM + 15) / 16;   // row tiles per workgroup (max)
  static constexpr int kLinW = D * D + D;            // one Linear's weight + bias
  static constexpr int kPartAttn = 4 * kLinW;        // the four Linears' partials
  __device__ __host__ static int nt(int M) { return (kGroups * M + 15) / 16; }
};
static_assert(AG<64>::NTmax <= kMaxM && AG<128>::NTmax == 3, "row tiles");

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Phase timestamps (diagnostic builds only, -DNCF_ATTN_STAMPS; tools/attn_stamps.py): thread 0
// of each workgroup records the shader clock at the phase boundaries of the block kernels.
#ifdef NCF_ATTN_STAMPS
__device__ unsigned long long g_attn_stamps[2][1024][16];
#define NCF_ASTAMP(dir, k)                                                                 \
  do {                                                                                     \
    if (threadIdx.x == 0) g_attn_stamps[dir][blockIdx.x & 1023][k] = clock64();           \
  } while (0)
#else
#define NCF_ASTAMP(dir, k) \
  do {                     \
  } while (0)
#endif

// acc += A[16 rows at X, D k] . B (B fragment: this lane's D/4 k values)
template <int D>
__device__ __forceinline__ f32x4 tile_mfma(const float* __restrict__ X, const float (&b)[D / 4],
                                           f32x4 acc) {
  constexpr int KF = D / 4;
  const int l = threadIdx.x & 63;
  const float* a = X + (l & 15) * AG<D>::kPitch + KF * (l >> 4);
  float av[KF];
#pragma unroll
  for (int q = 0; q < KF / 4; ++q) {
    const float4 v = *reinterpret_cast<const float4*>(a + 4 * q);
    av[4 * q] = v.x; av[4 * q + 1] = v.y; av[4 * q + 2] = v.z; av[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int s = 0; s < KF; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], b[s], acc, 0, 0, 0);
  return acc;
}

// B fragment of x W^T (forward): B[k][j] = W[j][k], j = 16w + (lane & 15), k = (D/4)g + s
template <int D>
__device__ __forceinline__ void frag_wt(const float* __restrict__ W, int w, float (&b)[D / 4]) {
  constexpr int KF = D / 4;
  const int l = threadIdx.x & 63;
  const float* p = W + (16 * w + (l & 15)) * D + KF * (l >> 4);
#pragma unroll
  for (int q = 0; q < KF / 4; ++q) {
    const float4 v = ld4(p + 4 * q);
    b[4 * q] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
  }
}

// B fragment of dz W (backward): B[k][j] = W[k][j], j = 16w + (lane & 15), k = (D/4)g + s
template <int D>
__device__ __forceinline__ void frag_w(const float* __restrict__ W, int w, float (&b)[D / 4]) {
  constexpr int KF = D / 4;
  const int l = threadIdx.x & 63;
  const float* p = W + (KF * (l >> 4)) * D + 16 * w + (l & 15);
#pragma unroll
  for (int s = 0; s < KF; ++s) b[s] = p[s * D];
}

// C fragment (rows 4g + r of the row tile, column 16w + (lane & 15)) -> LDS
template <int D>
__device__ __forceinline__ void put_tile(float* __restrict__ S, int rt, int w, f32x4 c) {
  constexpr int P = AG<D>::kPitch;
  const int l = threadIdx.x & 63;
  float* p = S + (16 * rt + 4 * (l >> 4)) * P + 16 * w + (l & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) p[r * P] = c[r];
}

// Fact 6: in training every group's M rows hold ONE user, so its M LayerNorm'd user
// rows are equal and so are their Q rows.  Whether every group of this workgroup has one user id
// (the caller's ids, uid[r0 ..]): then Q is projected for one row per group — the G group rows
// gathered into a single row tile — and copied back to all M rows of each group: the same bits
// as projecting every row (tested), one row tile of MFMA work instead of NT.  The test is also
// the staging barrier (__syncthreads_or).
__device__ __forceinline__ bool ids_uniform(const int64_t* __restrict__ uid, int ng, int M) {
  int diff = 0;
  for (int e = threadIdx.x; e < ng * (M - 1); e += blockDim.x) {
    const int gl = e / (M - 1), i = 1 + e % (M - 1);
    diff |= uid[gl * M + i] != uid[gl * M];
  }
  return __syncthreads_or(diff) == 0;
}

// The row holding row r's LayerNorm'd user row: with group_rows = M the gather
// (ncf_gather_ln_gmf_scaled_fwd) writes it only for a group's first row and for rows whose user
// differs from that row's; the others read the group's first row (the same bits).  (r < rows;
// the workgroup's rows start at a group boundary.)
// The per-workgroup record of the shared-Q decision, kept next to the stash: a forward that
// stashed Q once per group (at each group's first row) writes this word into the first column of
// the workgroup's second row, a row it never writes otherwise; a forward that stashed every row
// overwrites it with a projection (a NaN carrying this payload never comes out of one).  The stash
// backward reads the decision there instead of re-deciding it from the ids it is handed.
constexpr uint32_t kQGroupTag = 0x7FC0A51Bu;

__device__ __forceinline__ int src_row(const int64_t* __restrict__ uid, int r, int M) {
  if (!uid || M <= 1) return r;
  const int f = r - r % M;
  return (r == f || uid[r] != uid[f]) ? r : f;
}

// Rp rows of X_u into S (rows >= `rows` zero), each from its source row (src_row), every load in
// flight before the first LDS store
template <int D>
__device__ __forceinline__ void stage_in_src(float* __restrict__ S, const float* __restrict__ X,
                                             const int64_t* __restrict__ uid, int M, int Rp,
                                             int rows) {
  constexpr int L4 = D / 4, P = AG<D>::kPitch;
  constexpr int IT = (16 * AG<D>::NTmax * L4 + kThreads - 1) / kThreads;
  float4 v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int e = threadIdx.x + kThreads * it, r = e / L4, c = (e % L4) * 4;
    v[it] = (e < Rp * L4 && r < rows) ? ld4(X + (int64_t)src_row(uid, r, M) * D + c)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int e = threadIdx.x + kThreads * it;
    if (e < Rp * L4) *reinterpret_cast<float4*>(S + (e / L4) * P + (e % L4) * 4) = v[it];
  }
}

// group gl's first row (row gl M of X) -> row gl of Y, for the G groups of the workgroup
template <int D>
__device__ __forceinline__ void gather_group_rows(float* __restrict__ Y, const float* __restrict__ X,
                                                  int M) {
  constexpr int L4 = D / 4, P = AG<D>::kPitch;
  for (int e = threadIdx.x; e < AG<D>::kGroups * L4; e += blockDim.x) {
    const int gl = e / L4, c = (e % L4) * 4;
    *reinterpret_cast<float4*>(Y + gl * P + c) = *reinterpret_cast<const float4*>(X + gl * M * P + c);
  }
}

// row gl of Y -> rows gl M .. gl M + M - 1 of X for the Rp padded rows (rows >= zero_from: 0,
// the padded rows of the recompute backward), every thread a float4 at a time
template <int D>
__device__ __forceinline__ void expand_group_rows(float* __restrict__ X, const float* __restrict__ Y,
                                                  int M, int Rp, int zero_from) {
  constexpr int L4 = D / 4, P = AG<D>::kPitch;
  for (int e = threadIdx.x; e < Rp * L4; e += blockDim.x) {
    const int r = e / L4, c = (e % L4) * 4;
    const int gl = min(r / M, AG<D>::kGroups - 1);
    *reinterpret_cast<float4*>(X + r * P + c) =
        r < zero_from ? *reinterpret_cast<const float4*>(Y + gl * P + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Rp (padded) rows into LDS; rows >= `rows` are zeros
template <int D>
__device__ __forceinline__ void stage_in(float* __restrict__ S, const float* __restrict__ X,
                                         int Rp, int rows) {
  constexpr int L = D / 4;
  for (int e = threadIdx.x; e < Rp * L; e += blockDim.x) {
    const int r = e / L, c = (e % L) * 4;
    const float4 v = r < rows ? ld4(X + (int64_t)r * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(S + r * AG<D>::kPitch + c) = v;
  }
}

// NB [Rp x D] row blocks into LDS with every block's loads in flight before the first LDS
// store.  (A load-then-store loop waits one HBM latency per iteration: stamped at 12K cycles
// for the forward's two blocks and 20K for the backward's five, of 45K / 75K per workgroup.)
// Rows >= `rows` are zeros.
// Block `grp` (>= 0) is stored once per group (row gl M holds group gl's row, the forward's Q
// stash with one user per group): its rows are read from their group's first row.
template <int D, int NB>
__device__ __forceinline__ void stage_in_n(float* const (&S)[NB], const float* const (&X)[NB],
                                           int Rp, int rows, int grp = -1, int M = 1) {
  constexpr int L4 = D / 4, P = AG<D>::kPitch;
  constexpr int IT = (16 * AG<D>::NTmax * L4 + kThreads - 1) / kThreads;
  float4 v[NB][IT];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = threadIdx.x + kThreads * it, r = e / L4, c = (e % L4) * 4;
      const int src = b == grp ? r - r % M : r;
      v[b][it] = (e < Rp * L4 && r < rows) ? ld4(X[b] + (int64_t)src * D + c)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = threadIdx.x + kThreads * it;
      if (e < Rp * L4) *reinterpret_cast<float4*>(S[b] + (e / L4) * P + (e % L4) * 4) = v[b][it];
    }
}

template <int D>
__device__ __forceinline__ void stage_out(float* __restrict__ X, const float* __restrict__ S,
                                          int rows) {
  constexpr int L = D / 4;
  for (int e = threadIdx.x; e < rows * L; e += blockDim.x) {
    const int r = e / L, c = (e % L) * 4;
    st4(X + (int64_t)r * D + c, *reinterpret_cast<const float4*>(S + r * AG<D>::kPitch + c));
  }
}

// rows 0, M, 2M, .. (each group's first row) of S into X (the per-group Q stash)
template <int D>
__device__ __forceinline__ void stage_out_groups(float* __restrict__ X, const float* __restrict__ S,
                                                 int ng, int M) {
  constexpr int L = D / 4;
  for (int e = threadIdx.x; e < ng * L; e += blockDim.x) {
    const int r = (e / L) * M, c = (e % L) * 4;
    st4(X + (int64_t)r * D + c, *reinterpret_cast<const float4*>(S + r * AG<D>::kPitch + c));
  }
}

// whether row tile rt is this wave's (column slice w % CS, row tiles w / CS + RP j)
template <int D>
__device__ __forceinline__ bool my_tile(int rt, int NT) {
  return rt < NT && rt % AG<D>::RP == (int)(threadIdx.x >> 6) / AG<D>::CS;
}
template <int D>
__device__ __forceinline__ int my_slice() { return (int)(threadIdx.x >> 6) % AG<D>::CS; }

// out[rt] = X . W^T + bias for this wave's row tiles of its column slice, with the weight
// fragment b (frag_wt) and bias value bb already in registers
template <int D>
__device__ __forceinline__ void project_f(const float* __restrict__ X, const float (&b)[D / 4],
                                          float bb, int NT, f32x4 (&out)[kMaxM]) {
#pragma unroll
  for (int rt = 0; rt < AG<D>::NTmax; ++rt) {
    if (my_tile<D>(rt, NT)) {
      f32x4 acc = {bb, bb, bb, bb};
      out[rt] = tile_mfma<D>(X + 16 * rt * AG<D>::kPitch, b, acc);
    }
  }
}

// out[rt] = X . W^T + bias for this wave's row tiles of its column slice
template <int D>
__device__ __forceinline__ void project(const float* __restrict__ X, const float* __restrict__ W,
                                        const float* __restrict__ bias, int NT, f32x4 (&out)[kMaxM]) {
  const int w = my_slice<D>();
  float b[D / 4];
  frag_wt<D>(W, w, b);
  const float bb = bias ? bias[16 * w + (threadIdx.x & 15)] : 0.0f;
#pragma unroll
  for (int rt = 0; rt < AG<D>::NTmax; ++rt) {
    if (my_tile<D>(rt, NT)) {
      f32x4 acc = {bb, bb, bb, bb};
      // bias first, then the k chain: fmaf(..., bias) order of the unfused GEMM epilogue
      // differs only in rounding (tolerance-level)
      out[rt] = tile_mfma<D>(X + 16 * rt * AG<D>::kPitch, b, acc);
    }
  }
}

// Weight-gradient tiles of a Linear over this workgroup's rows: dW[a][b] = sum_r dY[r][a] X[r][b]
// (contraction over the Rp padded rows: k-permuted, lane group g covers rows [g Rp/4, (g+1)
// Rp/4)), written to out[D x D].  Rows past the batch are zero in LDS.
template <int D>
__device__ __forceinline__ void wgrad_tile(const float* __restrict__ dYs,
                                           const float* __restrict__ Xs, int Rp, int tj, int tk,
                                           float* __restrict__ out) {
  constexpr int P = AG<D>::kPitch;
  const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
  const int R4 = Rp >> 2;
  const float* a = dYs + (g * R4) * P + 16 * tj + i;
  const float* b = Xs + (g * R4) * P + 16 * tk + i;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 1 < R4; s += 2) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s * P], b[s * P], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(s + 1) * P], b[(s + 1) * P], acc1, 0, 0, 0);
  }
  if (s < R4) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s * P], b[s * P], acc0, 0, 0, 0);
  float* o = out + (16 * tj + 4 * g) * D + 16 * tk + i;
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r * D] = acc0[r] + acc1[r];
}

// bias gradient columns: out[c] = sum_r dY[r][c]; D threads per vector starting at thread t0
template <int D>
__device__ __forceinline__ void bias_cols(const float* __restrict__ dYs, int Rp, int t0,
                                          float* __restrict__ out) {
  const int c = (int)threadIdx.x - t0;
  if (c < 0 || c >= D) return;
  float acc = 0.0f;
  for (int r = 0; r < Rp; ++r) acc += dYs[r * AG<D>::kPitch + c];
  out[c] = acc;
}

// The per-group multi-head core of the forward, one lane per (group, head, query row), as
// k_attn_fwd (same P layout and dropout index (t*M + j) with t = (b*H + h)*M + i): softmax of
// Qs.Ks^T / scale, dropout on the weights, times Vs -> Os (rows in LDS, pitch kPitch).  The
// probabilities go to Pg (global, [B][H][M][M]) and/or Pl (LDS, [16][H][M][M]) when given.  Os
// may alias Qs: every lane finishes reading Q/K/V before the first store.  Shared by the forward
// and the backward's recompute, so both produce the same bits.
// Fact 6 form of the scores: with one user per group the M query rows of a group share Q, so a
// (group, head)'s scores Q K_j^T / scale are the same for all of them — computed once per (group,
// head, key j) into Sc[(gl H + h) M + j] with the core's own arithmetic (the same bits).
template <int D, int HD>
__device__ __forceinline__ void attn_scores_shared(const float* Qs, const float* Ks,
                                                   float* __restrict__ Sc, int ng, int M,
                                                   float scale) {
  constexpr int H = D / HD, kPitch = AG<D>::kPitch;
  for (int t = threadIdx.x; t < ng * H * M; t += kThreads) {
    const int j = t % M, h = (t / M) % H, gl = t / (M * H);
    const float* q = Qs + (gl * M) * kPitch + h * HD;   // (every row of the group holds it)
    const float* k = Ks + (gl * M + j) * kPitch + h * HD;
    float acc = 0.0f;
#pragma unroll
    for (int d = 0; d < HD; ++d) acc = fmaf(q[d], k[d], acc);
    Sc[t] = acc / scale;
  }
}

template <int D, int HD>
__device__ __forceinline__ void attn_core_fwd(const float* Qs, const float* Ks, const float* Vs,
                                              float* Os, float* Pl, float* __restrict__ Pg,
                                              int64_t g0, int ng, int M, float scale,
                                              float p_drop, uint64_t seed,
                                              const float* Sc = nullptr) {
  constexpr int H = D / HD, kPitch = AG<D>::kPitch;
  constexpr int kIt = (AG<D>::kGroups * H * kMaxM + kThreads - 1) / kThreads;
  const float inv_keep = p_drop > 0.0f ? 1.0f / (1.0f - p_drop) : 1.0f;
  const int ntask = ng * H * M;
  float o[kIt][HD];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + kThreads * it;
    if (t < ntask) {
      const int i = t % M, h = (t / M) % H, gl = t / (M * H);
      const int64_t tg = ((g0 + gl) * H + h) * M + i;
      const float* q = Qs + (gl * M + i) * kPitch + h * HD;
      float s[kMaxM];
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < kMaxM; ++j)
        if (j < M) {
          if (Sc) {
            s[j] = Sc[(gl * H + h) * M + j];
          } else {
            const float* k = Ks + (gl * M + j) * kPitch + h * HD;
            float acc = 0.0f;
#pragma unroll
            for (int d = 0; d < HD; ++d) acc = fmaf(q[d], k[d], acc);
            s[j] = acc / scale;
          }
          mx = fmaxf(mx, s[j]);
        }
      float sum = 0.0f;
#pragma unroll
      for (int j = 0; j < kMaxM; ++j)
        if (j < M) {
          s[j] = expf(s[j] - mx);
          sum += s[j];
        }
#pragma unroll
      for (int d = 0; d < HD; ++d) o[it][d] = 0.0f;
#pragma unroll
      for (int j = 0; j < kMaxM; ++j)
        if (j < M) {
          const float pj = s[j] / sum;
          if (Pg) Pg[tg * M + j] = pj;
          if (Pl) Pl[((gl * H + h) * M + i) * M + j] = pj;
          const float pd =
              p_drop > 0.0f ? pj * ncf_dropout_scale(seed, (uint64_t)tg * M + j, p_drop, inv_keep) : pj;
          const float* v = Vs + (gl * M + j) * kPitch + h * HD;
#pragma unroll
          for (int d = 0; d < HD; ++d) o[it][d] = fmaf(pd, v[d], o[it][d]);
        }
    }
  }
  __syncthreads();   // every lane is done reading Q/K/V
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int t = threadIdx.x + kThreads * it;
    if (t < ntask) {
      const int i = t % M, h = (t / M) % H, gl = t / (M * H);
      float* dst = Os + (gl * M + i) * kPitch + h * HD;
#pragma unroll
      for (int d = 0; d < HD; d += 4) *reinterpret_cast<float4*>(dst + d) = make_float4(o[it][d], o[it][d + 1], o[it][d + 2], o[it][d + 3]);
    }
  }
}

// O = dropout(P) V from the forward's stashed probabilities (Pg, the [G][H][M][M] layout of
// attn_core_fwd) and V in LDS: attn_core_fwd's own accumulation (the same pj, the same dropout
// stream, fmaf over j in order), so O has the forward's bits without the forward stashing it.
// Rows past the batch are left alone (the caller zeroes them).
template <int D, int HD>
__device__ __forceinline__ void attn_pv(const float* __restrict__ Pg, const float* Vs, float* Os,
                                        int64_t g0, int ng, int M, float p_drop, uint64_t seed) {
  constexpr int H = D / HD, kPitch = AG<D>::kPitch;
  const float inv_keep = p_drop > 0.0f ? 1.0f / (1.0f - p_drop) : 1.0f;
  const int ntask = ng * H * M;
  for (int t = threadIdx.x; t < ntask; t += kThreads) {
    const int i = t % M, h = (t / M) % H, gl = t / (M * H);
    const int64_t tg = ((g0 + gl) * H + h) * M + i;
    float o[HD];
#pragma unroll
    for (int d = 0; d < HD; ++d) o[d] = 0.0f;
#pragma unroll
    for (int j = 0; j < kMaxM; ++j)
      if (j < M) {
        const float pj = Pg[tg * M + j];
        const float pd =
            p_drop > 0.0f ? pj * ncf_dropout_scale(seed, (uint64_t)tg * M + j, p_drop, inv_keep) : pj;
        const float* v = Vs + (gl * M + j) * kPitch + h * HD;
#pragma unroll
        for (int d = 0; d < HD; ++d) o[d] = fmaf(pd, v[d], o[d]);
      }
    float* dst = Os + (gl * M + i) * kPitch + h * HD;
#pragma unroll
    for (int d = 0; d < HD; d += 4) *reinterpret_cast<float4*>(dst + d) = make_float4(o[d], o[d + 1], o[d + 2], o[d + 3]);
  }
}

// per-workgroup partial of the four Linear gradients, in the flat parameter order
// [q.weight | q.bias | k.weight | k.bias | v.weight | v.bias | out.weight | out.bias]
// (AG<D>::kPartAttn floats)

template <int D, int HD>
__device__ __forceinline__ void attn_block_fwd_body(
    float* __restrict__ lds,
    const float* __restrict__ xu, const float* __restrict__ xi, int64_t B, int M,
    const float* __restrict__ wq, const float* __restrict__ bq, const float* __restrict__ wk,
    const float* __restrict__ bk, const float* __restrict__ wv, const float* __restrict__ bv,
    const float* __restrict__ wo, const float* __restrict__ bo, float scale, float p_drop,
    uint64_t seed, const ncf_step_clock* clock, float* __restrict__ Q, float* __restrict__ K,
    float* __restrict__ V, float* __restrict__ P, float* __restrict__ O, float* __restrict__ Y,
    int core, const int64_t* __restrict__ uids, int share_q, float* __restrict__ Yl, int ypitch) {
  using G = AG<D>;
  constexpr int kPitch = G::kPitch;
  const int NT = G::nt(M), Rp = 16 * NT;
  float* S0 = lds;
  float* S1 = lds + Rp * kPitch;
  float* S2 = lds + 2 * Rp * kPitch;
  const int64_t g0 = (int64_t)blockIdx.x * G::kGroups;
  const int ng = (int)min<int64_t>(G::kGroups, B - g0);
  const int rows = ng * M;
  const int64_t r0 = g0 * M;
  const int w = my_slice<D>();
  // core == 0: eval with one item per group (softmax == 1, o = v).  Q/K/P/O may be NULL with
  // the core on: nothing is stashed (the backward recomputes it from X_u / X_i)
  if (clock) seed += clock->seed;

  NCF_ASTAMP(0, 0);
  // one user per group (fact 6): Q is projected from the G group rows of X_u, staged straight
  // into S2 (free until V lands) — the other M - 1 rows of each group are never read.  The
  // item rows' loads are in flight during the test (which is a barrier).
  bool shq = false;
  {
    constexpr int L4 = D / 4;
    constexpr int IT = (16 * G::NTmax * L4 + kThreads - 1) / kThreads;
    float4 vi[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = threadIdx.x + kThreads * it, r = e / L4, c = (e % L4) * 4;
      vi[it] = (e < Rp * L4 && r < rows) ? ld4(xi + (r0 + r) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (share_q && core && M > 1 && uids) shq = ids_uniform(uids + r0, ng, M);
    if (shq) {
      for (int e = threadIdx.x; e < G::kGroups * L4; e += kThreads) {
        const int gl = e / L4, c = (e % L4) * 4;
        const float4 v = gl < ng ? ld4(xu + (r0 + (int64_t)gl * M) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(S2 + gl * kPitch + c) = v;
      }
    } else if (core) {
      stage_in_src<D>(S0, xu + r0 * D, uids ? uids + r0 : nullptr, M, Rp, rows);
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = threadIdx.x + kThreads * it;
      if (e < Rp * L4) *reinterpret_cast<float4*>(S1 + (e / L4) * kPitch + (e % L4) * 4) = vi[it];
    }
  }
  // the projections' weight fragments of this wave's column slice, issued behind the rows' loads
  // (in flight during the staging barrier instead of in front of each projection); out_proj's
  // is loaded ahead of the core
  const int cl = 16 * w + (threadIdx.x & 15);
  float fw_v[D / 4], fw_q[D / 4], fw_k[D / 4], fw_o[D / 4];
  frag_wt<D>(wv, w, fw_v);
  const float bb_v = bv ? bv[cl] : 0.0f, bb_o = bo ? bo[cl] : 0.0f;
  float bb_q = 0.0f, bb_k = 0.0f;
  if (core) {
    frag_wt<D>(wq, w, fw_q);
    frag_wt<D>(wk, w, fw_k);
    bb_q = bq ? bq[cl] : 0.0f;
    bb_k = bk ? bk[cl] : 0.0f;
  }
  __syncthreads();
  NCF_ASTAMP(0, 1);
  if (!core) frag_wt<D>(wo, w, fw_o);
  f32x4 fq[kMaxM], fk[kMaxM], fv[kMaxM];
  project_f<D>(S1, fw_v, bb_v, NT, fv);
  if (core) {
    if (shq)
      project_f<D>(S2, fw_q, bb_q, 1, fq);
    else
      project_f<D>(S0, fw_q, bb_q, NT, fq);
    project_f<D>(S1, fw_k, bb_k, NT, fk);
  }
  __syncthreads();
  NCF_ASTAMP(0, 2);
  float* Qx = S2 + Rp * kPitch + G::kGroups * 8 * kMaxM;   // [16][pitch] group-row Q tile
#pragma unroll
  for (int rt = 0; rt < G::NTmax; ++rt)
    if (my_tile<D>(rt, NT)) {
      put_tile<D>(S2, rt, w, fv[rt]);
      if (core) {
        if (!shq) put_tile<D>(S0, rt, w, fq[rt]);
        put_tile<D>(S1, rt, w, fk[rt]);
      }
    }
  if (shq && my_tile<D>(0, 1)) put_tile<D>(Qx, 0, w, fq[0]);
  __syncthreads();
  if (shq) {
    expand_group_rows<D>(S0, Qx, M, Rp, 1 << 30);
    __syncthreads();
  }
  NCF_ASTAMP(0, 3);
  const float* src = S2;   // the out_proj input: O, or V when there is no core
  if (core) {
    // (one user per group: Q is stashed once per group, at the group's first row, and the
    // decision recorded beside it; the backward reads both there)
    if (Q) {
      if (shq) {
        stage_out_groups<D>(Q + r0 * D, S0, ng, M);
        if (threadIdx.x == 0) reinterpret_cast<uint32_t*>(Q)[(r0 + 1) * D] = kQGroupTag;
      } else {
        stage_out<D>(Q + r0 * D, S0, rows);
      }
    }
    if (K) stage_out<D>(K + r0 * D, S1, rows);
    if (V) stage_out<D>(V + r0 * D, S2, rows);
    NCF_ASTAMP(0, 4);
    float* Sc = S2 + Rp * kPitch;   // [G][H][M] shared scores (past the three row buffers)
    frag_wt<D>(wo, w, fw_o);        // (lands during the core)
    if (shq) {
      attn_scores_shared<D, HD>(S0, S1, Sc, ng, M, scale);
      __syncthreads();
    }
    attn_core_fwd<D, HD>(S0, S1, S2, S0, nullptr, P, g0, ng, M, scale, p_drop, seed,
                         shq ? Sc : nullptr);
    __syncthreads();
    NCF_ASTAMP(0, 5);
    if (O) stage_out<D>(O + r0 * D, S0, rows);
    src = S0;
  } else if (V) {
    stage_out<D>(V + r0 * D, S2, rows);
  }
  // out_proj -> S1 (K is dead) -> Y
  f32x4 fy[kMaxM];
  project_f<D>(src, fw_o, bb_o, NT, fy);
#pragma unroll
  for (int rt = 0; rt < G::NTmax; ++rt)
    if (my_tile<D>(rt, NT)) put_tile<D>(S1, rt, w, fy[rt]);
  __syncthreads();
  NCF_ASTAMP(0, 6);
  stage_out<D>(Y + r0 * D, S1, rows);
  if (Yl) {   // (fused with the tower: Y also into the tower's input tile, padding rows zero)
    constexpr int L4 = D / 4;
    const int Rp = 16 * G::nt(M);
    for (int e = threadIdx.x; e < Rp * L4; e += kThreads) {
      const int r = e / L4, c = (e % L4) * 4;
      *reinterpret_cast<float4*>(Yl + r * ypitch + c) =
          r < rows ? *reinterpret_cast<const float4*>(S1 + r * kPitch + c)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#ifdef NCF_ATTN_STAMPS
  __syncthreads();
#endif
  NCF_ASTAMP(0, 7);
}

template <int D, int HD>
__global__ __launch_bounds__(kThreads) void k_attn_block_fwd(
    const float* __restrict__ xu, const float* __restrict__ xi, int64_t B, int M,
    const float* __restrict__ wq, const float* __restrict__ bq, const float* __restrict__ wk,
    const float* __restrict__ bk, const float* __restrict__ wv, const float* __restrict__ bv,
    const float* __restrict__ wo, const float* __restrict__ bo, float scale, float p_drop,
    uint64_t seed, const ncf_step_clock* clock, float* __restrict__ Q, float* __restrict__ K,
    float* __restrict__ V, float* __restrict__ P, float* __restrict__ O, float* __restrict__ Y,
    int core, const int64_t* __restrict__ uids, int share_q) {
  extern __shared__ float lds[];
  attn_block_fwd_body<D, HD>(lds, xu, xi, B, M, wq, bq, wk, bk, wv, bv, wo, bo, scale, p_drop,
                             seed, clock, Q, K, V, P, O, Y, core, uids, share_q, nullptr, 0);
}

// RC (recompute): nothing was stashed by the forward.  Q, K, V are re-projected from X_u / X_i
// and the core forward (P, O) re-run in LDS with the forward's own code (attn_core_fwd: the same
// bits), instead of reading 4 stashed [rows][64] blocks and P back from HBM.
template <int D, int HD, bool RC, bool PF_OK = true>
__device__ __forceinline__ void attn_block_bwd_body(
    float* __restrict__ lds,
    const float* __restrict__ dY, const float* __restrict__ Qg, const float* __restrict__ Kg,
    const float* __restrict__ Vg, const float* __restrict__ Pg, int64_t B, int M,
    const float* __restrict__ wq, const float* __restrict__ wk, const float* __restrict__ wv,
    const float* __restrict__ wo, float scale, float p_drop, uint64_t seed,
    const ncf_step_clock* clock, const float* __restrict__ Og, const float* __restrict__ Xu,
    const float* __restrict__ Xi, float* __restrict__ part, float* __restrict__ dQ,
    float* __restrict__ dK, float* __restrict__ dV, float* __restrict__ dXu,
    float* __restrict__ dXi, const float* __restrict__ bq, const float* __restrict__ bk,
    const float* __restrict__ bv, const int64_t* __restrict__ uids, int share_q, const float* __restrict__ dYl, int dypitch) {
  using G = AG<D>;
  constexpr int kPitch = G::kPitch, kGroups = G::kGroups, kLinW = G::kLinW, L4 = D / 4;
  constexpr int H = D / HD;
  constexpr int kIt = (kGroups * H * kMaxM + kThreads - 1) / kThreads;
  const int NT = G::nt(M), Rp = 16 * NT;
  float* S0 = lds;
  float* S1 = lds + Rp * kPitch;
  float* S2 = lds + 2 * Rp * kPitch;
  float* S3 = lds + 3 * Rp * kPitch;
  const bool wg = RC || part != nullptr;   // fused weight gradients (partials of this workgroup)
  float* S4 = lds + 4 * Rp * kPitch;                // O -> X_u (fused weight gradients only)
  float* dS = lds + (wg ? 5 : 4) * Rp * kPitch;     // [G][H][M][M]
  float* Pl = dS + kGroups * H * M * M;             // RC: the recomputed P, same layout
  const int64_t g0 = (int64_t)blockIdx.x * kGroups;
  const int ng = (int)min<int64_t>(kGroups, B - g0);
  const int rows = ng * M;
  const int64_t r0 = g0 * M;
  const int w = my_slice<D>();
  if (clock) seed += clock->seed;
  const float inv_keep = p_drop > 0.0f ? 1.0f / (1.0f - p_drop) : 1.0f;

  NCF_ASTAMP(1, 0);
  // the stash form at D = 64 (hd <= 32: registers to spare) loads its four weight fragments
  // behind the rows' loads, so they land during the staging barrier
  // (PF_OK = false: fused behind the tower backward, tower_fused.hip, where the 64 registers of
  // the four fragments would lift the whole kernel's allocation)
  constexpr bool PF = PF_OK && !RC && D == 64 && HD <= 32;
  float pw_o[D / 4], pw_q[D / 4], pw_k[D / 4], pw_v[D / 4];
  constexpr int kPre = (16 * G::NTmax * L4 + kThreads - 1) / kThreads;   // float4 per thread
  float4 pu[kPre], pi[kPre];   // X_u / X_i rows for the fused weight gradients
  bool shq_src = false;        // (stash form) one user per group: X_u from the group rows
  if constexpr (RC) {
    // one user per group (the forward's test on the same ids: the same Q bits): only the G
    // group rows of X_u are read, straight into S3 (the Q projection's input)
    bool shq = false;
    {
      constexpr int IT = (16 * G::NTmax * L4 + kThreads - 1) / kThreads;
      float4 v0[IT], v2[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int e = threadIdx.x + kThreads * it, r = e / L4, c = (e % L4) * 4;
        const bool in = e < Rp * L4 && r < rows;
        v0[it] = in ? ld4(dY + (r0 + r) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        v2[it] = in ? ld4(Xi + (r0 + r) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (share_q && M > 1 && uids) shq = ids_uniform(uids + r0, ng, M);
      if (shq) {
        for (int e = threadIdx.x; e < kGroups * L4; e += kThreads) {
          const int gl = e / L4, c = (e % L4) * 4;
          const float4 v = gl < ng ? ld4(Xu + (r0 + (int64_t)gl * M) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(S3 + gl * kPitch + c) = v;
        }
      } else {
        stage_in_src<D>(S1, Xu + r0 * D, uids ? uids + r0 : nullptr, M, Rp, rows);
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int e = threadIdx.x + kThreads * it;
        if (e < Rp * L4) {
          *reinterpret_cast<float4*>(S0 + (e / L4) * kPitch + (e % L4) * 4) = v0[it];
          *reinterpret_cast<float4*>(S2 + (e / L4) * kPitch + (e % L4) * 4) = v2[it];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPre; ++q) {   // (zero rows past the batch: staged as zeros)
      const int e = threadIdx.x + kThreads * q, r = e / L4, c = (e % L4) * 4;
      const bool in = e < Rp * L4;
      // X_u of row r: its group's row (shq) or its own
      const float* xu_r = shq ? S3 + min(r / M, kGroups - 1) * kPitch + c : S1 + r * kPitch + c;
      pu[q] = in && (!shq || r < rows) ? *reinterpret_cast<const float4*>(xu_r)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
      pi[q] = in ? *reinterpret_cast<const float4*>(S2 + r * kPitch + c)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    f32x4 fq[kMaxM], fk[kMaxM], fv[kMaxM];
    if (shq)
      project<D>(S3, wq, bq, 1, fq);
    else
      project<D>(S1, wq, bq, NT, fq);
    project<D>(S2, wk, bk, NT, fk);
    project<D>(S2, wv, bv, NT, fv);
    __syncthreads();
    // rows past the batch (a ragged last workgroup) hold zeros, as the stashing form stages
    // them: the bias columns of dQ/dK/dV later sum over all R rows of these buffers
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    const int rsub = 4 * ((threadIdx.x & 63) >> 4);
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) {
        const bool pad = 16 * rt + rsub + 3 >= rows;
        f32x4 a = fq[rt], b = fk[rt], c = fv[rt];
        if (pad) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (16 * rt + rsub + e >= rows) { a[e] = 0.f; b[e] = 0.f; c[e] = 0.f; }
        }
        if (!shq) put_tile<D>(S1, rt, w, a);
        put_tile<D>(S2, rt, w, b);
        put_tile<D>(S3, rt, w, c);
        if (16 * rt + rsub + 3 >= rows) put_tile<D>(S4, rt, w, z4);   // O of padded rows
      }
    float* Qx = Pl + kGroups * H * M * M;   // [16][pitch] group-row Q tile
    if (shq && my_tile<D>(0, 1)) put_tile<D>(Qx, 0, w, fq[0]);
    __syncthreads();
    if (shq) {
      expand_group_rows<D>(S1, Qx, M, Rp, rows);
      __syncthreads();
    }
    attn_core_fwd<D, HD>(S1, S2, S3, S4, Pl, nullptr, g0, ng, M, scale, p_drop, seed);
  } else {
    // the forward stashed Q once per group where every group of the workgroup holds one user,
    // and recorded that next to the stash (kQGroupTag); block 1 (Q) is then read from the group
    // rows.  (share_q is unused here: the record, not the ids handed to the backward, decides.)
    const bool shq = M > 1 && Qg &&
                     __float_as_uint(Qg[(r0 + 1) * D]) == kQGroupTag;
    shq_src = shq;
    if (wg && Og) {
      float* const dst[5] = {S0, S1, S2, S3, S4};
      const float* const src[5] = {dY + r0 * D, Qg + r0 * D, Kg + r0 * D, Vg + r0 * D,
                                   Og + r0 * D};
      stage_in_n<D, 5>(dst, src, Rp, rows, shq ? 1 : -1, M);
    } else if (wg && dYl) {
      // fused behind the tower backward (tower_fused.hip): dY is that kernel's dX tile in LDS
      // (it overlaps S3/S4: copied into S0 first, one barrier, then the stash's rows); O not
      // stashed: recomputed from the stashed P and V as below
      for (int e = threadIdx.x; e < Rp * L4; e += kThreads) {
        const int r = e / L4, c = (e % L4) * 4;
        *reinterpret_cast<float4*>(S0 + r * kPitch + c) =
            r < rows ? *reinterpret_cast<const float4*>(dYl + r * dypitch + c)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      __syncthreads();
      float* const dst[3] = {S1, S2, S3};
      const float* const src[3] = {Qg + r0 * D, Kg + r0 * D, Vg + r0 * D};
      stage_in_n<D, 3>(dst, src, Rp, rows, shq ? 0 : -1, M);
      for (int e = threadIdx.x; e < (Rp - rows) * L4; e += kThreads)   // padded rows: zeros
        *reinterpret_cast<float4*>(S4 + (rows + e / L4) * kPitch + (e % L4) * 4) =
            make_float4(0.f, 0.f, 0.f, 0.f);
      __syncthreads();
      attn_pv<D, HD>(Pg, S3, S4, g0, ng, M, p_drop, seed);
    } else if (wg) {
      // O not stashed: recomputed from the stashed P and V (attn_pv: the forward's bits)
      float* const dst[4] = {S0, S1, S2, S3};
      const float* const src[4] = {dY + r0 * D, Qg + r0 * D, Kg + r0 * D, Vg + r0 * D};
      stage_in_n<D, 4>(dst, src, Rp, rows, shq ? 1 : -1, M);
      for (int e = threadIdx.x; e < (Rp - rows) * L4; e += kThreads)   // padded rows: zeros
        *reinterpret_cast<float4*>(S4 + (rows + e / L4) * kPitch + (e % L4) * 4) =
            make_float4(0.f, 0.f, 0.f, 0.f);
      __syncthreads();
      attn_pv<D, HD>(Pg, S3, S4, g0, ng, M, p_drop, seed);
    } else {
      float* const dst[4] = {S0, S1, S2, S3};
      const float* const src[4] = {dY + r0 * D, Qg + r0 * D, Kg + r0 * D, Vg + r0 * D};
      stage_in_n<D, 4>(dst, src, Rp, rows, shq ? 1 : -1, M);
    }
  }
  if constexpr (PF) {
    frag_w<D>(wo, w, pw_o);
    frag_w<D>(wq, w, pw_q);
    frag_w<D>(wk, w, pw_k);
    frag_w<D>(wv, w, pw_v);
  }
  __syncthreads();
  NCF_ASTAMP(1, 1);
  float* pw = wg ? part + (int64_t)blockIdx.x * G::kPartAttn : nullptr;
  // X_u / X_i rows of this workgroup, prefetched into registers for the fused weight gradients
  if (wg && !RC) {
#pragma unroll
    for (int q = 0; q < kPre; ++q) {
      const int e = threadIdx.x + kThreads * q, r = e / L4, c = (e % L4) * 4;
      const bool in = e < Rp * L4 && r < rows;
      // (a shared-Q workgroup holds one user per group: its group's first row)
      const int sr = !in ? 0 : shq_src ? r - r % M : src_row(uids ? uids + r0 : nullptr, r, M);
      pu[q] = in ? ld4(Xu + (r0 + sr) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      pi[q] = in ? ld4(Xi + (r0 + r) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // dO = dY . Wo  (+ out_proj's weight gradient dY^T O and bias gradient)
  {
    float b[D / 4];
    if constexpr (PF) {
#pragma unroll
      for (int s = 0; s < D / 4; ++s) b[s] = pw_o[s];
    } else {
      frag_w<D>(wo, w, b);
    }
    f32x4 fo[kMaxM];
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) fo[rt] = tile_mfma<D>(S0 + 16 * rt * kPitch, b, f32x4{0.f, 0.f, 0.f, 0.f});
    if (wg) {
      const int wave = threadIdx.x >> 6;
#pragma unroll
      for (int q = 0; q < G::CS * G::CS / 8; ++q) {   // the D/16 x D/16 tiles over 8 waves
        const int t = wave + 8 * q;
        wgrad_tile<D>(S0, S4, Rp, t / G::CS, t % G::CS, pw + 3 * kLinW);
      }
      bias_cols<D>(S0, Rp, 0, pw + 3 * kLinW + D * D);
    }
    __syncthreads();
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) put_tile<D>(S0, rt, w, fo[rt]);
    if (wg) {   // O is consumed: X_u takes its place
#pragma unroll
      for (int q = 0; q < kPre; ++q) {
        const int e = threadIdx.x + kThreads * q;
        if (e < Rp * L4) *reinterpret_cast<float4*>(S4 + (e / L4) * kPitch + (e % L4) * 4) = pu[q];
      }
    }
    __syncthreads();
  }
  NCF_ASTAMP(1, 2);
  const int ntask = ng * H * M;
  // core, query side (as k_attn_bwd_q): dS and dQ per (group, head, query row)
  {
    float dq[kIt][HD];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = threadIdx.x + kThreads * it;
      if (t < ntask) {
        const int i = t % M, h = (t / M) % H, gl = t / (M * H);
        const int64_t tg = ((g0 + gl) * H + h) * M + i;
        const float* go = S0 + (gl * M + i) * kPitch + h * HD;
        const float* prow = RC ? Pl + ((gl * H + h) * M + i) * M : Pg + tg * M;
        float dp[kMaxM], pr[kMaxM];
        float tsum = 0.0f;
#pragma unroll
        for (int j = 0; j < kMaxM; ++j)
          if (j < M) {
            const float* v = S3 + (gl * M + j) * kPitch + h * HD;
            float acc = 0.0f;
#pragma unroll
            for (int d = 0; d < HD; ++d) acc = fmaf(go[d], v[d], acc);
            if (p_drop > 0.0f) acc *= ncf_dropout_scale(seed, (uint64_t)tg * M + j, p_drop, inv_keep);
            dp[j] = acc;
            pr[j] = prow[j];
            tsum = fmaf(pr[j], acc, tsum);
          }
#pragma unroll
        for (int d = 0; d < HD; ++d) dq[it][d] = 0.0f;
        float* dsrow = dS + ((gl * H + h) * M + i) * M;
#pragma unroll
        for (int j = 0; j < kMaxM; ++j)
          if (j < M) {
            const float ds = pr[j] * (dp[j] - tsum);
            dsrow[j] = ds;
            const float* k = S2 + (gl * M + j) * kPitch + h * HD;
#pragma unroll
            for (int d = 0; d < HD; ++d) dq[it][d] = fmaf(ds, k[d], dq[it][d]);
          }
      }
    }
    __syncthreads();   // K, V no longer read; dS complete
    NCF_ASTAMP(1, 3);
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = threadIdx.x + kThreads * it;
      if (t < ntask) {
        const int i = t % M, h = (t / M) % H, gl = t / (M * H);
        float* dst = S2 + (gl * M + i) * kPitch + h * HD;
#pragma unroll
        for (int d = 0; d < HD; ++d) dst[d] = dq[it][d] / scale;
      }
    }
  }
  // core, key side (as k_attn_bwd_kv): dK, dV per (group, head, key row)
  {
    float dk[kIt][HD];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = threadIdx.x + kThreads * it;
      if (t < ntask) {
        const int j = t % M, h = (t / M) % H, gl = t / (M * H);
        float dv[HD];
#pragma unroll
        for (int d = 0; d < HD; ++d) { dk[it][d] = 0.0f; dv[d] = 0.0f; }
        const int64_t bh = (g0 + gl) * H + h;
        for (int i = 0; i < M; ++i) {
          const int64_t row = bh * M + i;
          const float ds = dS[((gl * H + h) * M + i) * M + j];
          float pd = RC ? Pl[((gl * H + h) * M + i) * M + j] : Pg[row * M + j];
          if (p_drop > 0.0f) pd *= ncf_dropout_scale(seed, (uint64_t)row * M + j, p_drop, inv_keep);
          const float* q = S1 + (gl * M + i) * kPitch + h * HD;
          const float* go = S0 + (gl * M + i) * kPitch + h * HD;
#pragma unroll
          for (int d = 0; d < HD; ++d) {
            dk[it][d] = fmaf(ds, q[d], dk[it][d]);
            dv[d] = fmaf(pd, go[d], dv[d]);
          }
        }
        float* dst = S3 + (gl * M + j) * kPitch + h * HD;   // V is dead
#pragma unroll
        for (int d = 0; d < HD; ++d) dst[d] = dv[d];
      }
    }
    __syncthreads();   // Q no longer read
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = threadIdx.x + kThreads * it;
      if (t < ntask) {
        const int j = t % M, h = (t / M) % H, gl = t / (M * H);
        float* dst = S1 + (gl * M + j) * kPitch + h * HD;
#pragma unroll
        for (int d = 0; d < HD; ++d) dst[d] = dk[it][d] / scale;
      }
    }
    __syncthreads();
  }
  NCF_ASTAMP(1, 4);
  if (dQ) stage_out<D>(dQ + r0 * D, S2, rows);
  if (dK) stage_out<D>(dK + r0 * D, S1, rows);
  if (dV) stage_out<D>(dV + r0 * D, S3, rows);
  if (wg) {   // dO is consumed: X_i takes its place; then the q/k/v weight gradients
#pragma unroll
    for (int q = 0; q < kPre; ++q) {
      const int e = threadIdx.x + kThreads * q;
      if (e < Rp * L4) *reinterpret_cast<float4*>(S0 + (e / L4) * kPitch + (e % L4) * 4) = pi[q];
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    constexpr int TPL = G::CS * G::CS;   // 16x16 tiles per weight
    for (int q = 0; q < 3 * TPL / 8; ++q) {
      const int t = wave + 8 * q, lin = t / TPL, tt = t % TPL;   // lin: 0 q, 1 k, 2 v
      const float* dys = lin == 0 ? S2 : (lin == 1 ? S1 : S3);
      const float* xs = lin == 0 ? S4 : S0;
      wgrad_tile<D>(dys, xs, Rp, tt / G::CS, tt % G::CS, pw + lin * kLinW);
    }
    bias_cols<D>(S2, Rp, 0, pw + D * D);
    bias_cols<D>(S1, Rp, D, pw + kLinW + D * D);
    bias_cols<D>(S3, Rp, 2 * D, pw + 2 * kLinW + D * D);
  }
  NCF_ASTAMP(1, 5);
  // dX_u = dQ . Wq ; dX_i = dK . Wk + dV . Wv
  f32x4 fu[kMaxM], fi[kMaxM];
  if constexpr (PF) {
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) fu[rt] = tile_mfma<D>(S2 + 16 * rt * kPitch, pw_q, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) fi[rt] = tile_mfma<D>(S1 + 16 * rt * kPitch, pw_k, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) fi[rt] = tile_mfma<D>(S3 + 16 * rt * kPitch, pw_v, fi[rt]);
  } else {
    float b[D / 4];
    frag_w<D>(wq, w, b);
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) fu[rt] = tile_mfma<D>(S2 + 16 * rt * kPitch, b, f32x4{0.f, 0.f, 0.f, 0.f});
    frag_w<D>(wk, w, b);
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) fi[rt] = tile_mfma<D>(S1 + 16 * rt * kPitch, b, f32x4{0.f, 0.f, 0.f, 0.f});
    frag_w<D>(wv, w, b);
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) fi[rt] = tile_mfma<D>(S3 + 16 * rt * kPitch, b, fi[rt]);
  }
  if (!wg) {
#pragma unroll
    for (int rt = 0; rt < G::NTmax; ++rt)
      if (my_tile<D>(rt, NT)) put_tile<D>(S0, rt, w, fu[rt]);   // dO is dead
  }
  __syncthreads();   // S0..S4 no longer read (MFMA operands, stage_out)
  NCF_ASTAMP(1, 6);
#pragma unroll
  for (int rt = 0; rt < G::NTmax; ++rt)
    if (my_tile<D>(rt, NT)) {
      if (wg) put_tile<D>(S0, rt, w, fu[rt]);
      put_tile<D>(S1, rt, w, fi[rt]);
    }
  __syncthreads();
  NCF_ASTAMP(1, 7);
  stage_out<D>(dXu + r0 * D, S0, rows);
  stage_out<D>(dXi + r0 * D, S1, rows);
#ifdef NCF_ATTN_STAMPS
  __syncthreads();
#endif
  NCF_ASTAMP(1, 8);
}

template <int D, int HD, bool RC>
__global__ __launch_bounds__(kThreads) void k_attn_block_bwd(
    const float* __restrict__ dY, const float* __restrict__ Qg, const float* __restrict__ Kg,
    const float* __restrict__ Vg, const float* __restrict__ Pg, int64_t B, int M,
    const float* __restrict__ wq, const float* __restrict__ wk, const float* __restrict__ wv,
    const float* __restrict__ wo, float scale, float p_drop, uint64_t seed,
    const ncf_step_clock* clock, const float* __restrict__ Og, const float* __restrict__ Xu,
    const float* __restrict__ Xi, float* __restrict__ part, float* __restrict__ dQ,
    float* __restrict__ dK, float* __restrict__ dV, float* __restrict__ dXu,
    float* __restrict__ dXi, const float* __restrict__ bq, const float* __restrict__ bk,
    const float* __restrict__ bv, const int64_t* __restrict__ uids, int share_q) {
  extern __shared__ float lds[];
  attn_block_bwd_body<D, HD, RC>(lds, dY, Qg, Kg, Vg, Pg, B, M, wq, wk, wv, wo, scale, p_drop, seed,
                                 clock, Og, Xu, Xi, part, dQ, dK, dV, dXu, dXi, bq, bk, bv, uids,
                                 share_q, nullptr, 0);
}

// LDS per workgroup (gfx950: 160 KB) available to the dynamic buffers: the kernels' static LDS
// (the workgroup vote of groups_uniform) takes a few bytes of it
constexpr size_t kMaxLds = 160 * 1024 - 1024;
template <int D>
size_t fwd_lds(int M) {   // three row buffers + the shared scores [G][H <= 8][M] + the Q tile
  return sizeof(float) * (3 * 16 * AG<D>::nt(M) * AG<D>::kPitch + AG<D>::kGroups * 8 * kMaxM +
                          16 * AG<D>::kPitch);
}
template <int D>
size_t bwd_lds(int M, int H, bool wg, bool rc = false) {
  using G = AG<D>;
  return sizeof(float) * ((wg ? 5 : 4) * 16 * G::nt(M) * G::kPitch +
                          (rc ? 2 : 1) * G::kGroups * H * M * M + (rc ? 16 * G::kPitch : 0));
}
size_t fwd_lds_d(int D, int M) { return D == 64 ? fwd_lds<64>(M) : fwd_lds<128>(M); }
size_t bwd_lds_d(int D, int M, int H, bool wg, bool rc = false) {
  return D == 64 ? bwd_lds<64>(M, H, wg, rc) : bwd_lds<128>(M, H, wg, rc);
}
int groups_per_wg(int64_t D) { return D == 64 ? AG<64>::kGroups : AG<128>::kGroups; }
int64_t part_floats(int64_t D) { return D == 64 ? AG<64>::kPartAttn : AG<128>::kPartAttn; }

template <typename Kern>
void allow_lds(Kern k, size_t bytes) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// Q from one row per group when the groups hold one user each (ids_uniform; checked per
// workgroup on the device from the caller's ids): always on when user_ids are given (the engine's
// per-row A/B passes NULL ids with every row gathered, engine.ATTN_SHARE_Q).  The stash backward
// takes the forward's recorded decision (kQGroupTag), not its own.
constexpr int kShareQ = 1;

// head widths the kernels are built for: hd in {8, 16, 32, 64} at D = 64, {16, 32, 64} at
// D = 128 (the core keeps a head row of hd floats per lane in registers)
bool hd_ok(int64_t dim, int64_t hd) {
  if (dim == 64) return hd == 8 || hd == 16 || hd == 32 || hd == 64;
  return hd == 16 || hd == 32 || hd == 64;
}

// the per-workgroup partial rows -> the 8 parameter gradients: one reduction when they are laid
// out like the partial row (the flat gradient buffer), else one per Linear (weight + bias
// adjacent) or 8; deferred into `defer` when given
int defer_partials(int64_t D, float* const* grad_params, const float* part, int nb,
                   float* workspace, int64_t workspace_floats, ncf_reduce_list* defer,
                   void* stream) {
  const int64_t PA = part_floats(D), LW = D * D + D, DD = D * D;
  ncf_reduce_list local;
  local.count = 0;
  ncf_reduce_list* lst = defer ? defer : &local;
  int rc = NCF_OK;
  bool flat = true;
  for (int j = 1; j < 8; ++j)
    flat = flat && grad_params[j] == grad_params[0] + (j / 2) * LW + (j & 1) * DD;
  if (flat) {
    rc = ncf_defer(lst, part, nb, PA, PA, grad_params[0], 0, PA, PA);
  } else {
    for (int lin = 0; lin < 4 && !rc; ++lin) {
      float* gw = grad_params[2 * lin];
      float* gb = grad_params[2 * lin + 1];
      const float* pp = part + lin * LW;
      if (gb == gw + DD) {
        rc = ncf_defer(lst, pp, nb, PA, LW, gw, 0, LW, LW);
      } else {
        rc = ncf_defer(lst, pp, nb, PA, DD, gw, 0, DD, DD);
        if (!rc) rc = ncf_defer(lst, pp + DD, nb, PA, D, gb, 0, D, D);
      }
    }
  }
  if (rc) return rc;
  if (!defer) {
    const int64_t off = (int64_t)nb * PA;
    return ncf_reduce_batch(lst, workspace + off, workspace_floats - off, stream);
  }
  return NCF_OK;
}
}  // namespace
}  // namespace ncf_attn
