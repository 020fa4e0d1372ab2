// The MLP tower of AdvancedNCF in one launch per direction: 3 x [Linear -> ReLU -> LayerNorm ->
// Dropout] (+ mlp_output and the final fusion in the forward), for input width K0 = 64 (C2) or
// 128 (C4: mlp_embedding_dim = 128) and hidden widths [256, 128, 64] (the reference defaults).
//
// Reference: self.mlp (src/model/architecture.py:230-242, applied :344), mlp_output (:246, :345),
// final Linear(2,1) + Sigmoid (:249-252, :353-354).  Same math and dropout stream as the
// unfused path (GEMM with ReLU epilogue + rowops.hip + head.hip): LayerNorm of the ReLU output
// with the two-pass mean/variance, dropout keep decisions from ncf_dropout_scale4 at element
// index row*W + col with the per-layer seed (seed + 0x9E37*(l+1)) & (2^63-1) (+ the step clock).
// Only the fmaf order of the Linear layers (k-permuted MFMA below) differs.
//
// Tiling: a 512-thread workgroup (8 waves) owns kRows = 80 rows (5 MFMA row tiles) for the whole
// tower; the rows live in LDS between layers (buffers Q [80][260] and P [80][132], 125 KB: one
// workgroup per CU, 256 of them at 20,480 rows).  Row ops run in place; a layer's output goes to
// the other buffer.
//  * Linear: 16x16 output tiles of v_mfma_f32_16x16x4_f32.  A wave loads each weight chunk
//    (4 k-steps of its column) once from L2 and feeds all its row tiles with it (independent
//    accumulators): every weight byte serves 80 rows (~40 flop/B), where a 16-row tile left the
//    Linear phases bound by L2 weight traffic.  k-permuted operands: in MFMA step s lane group
//    g = lane>>4 supplies k = g*K/4 + s, so a lane's A row slice (LDS) and weight row slice are
//    contiguous float4 runs.
//  * Row ops: 16 lanes per row, width/64 float4 chunks per lane (the column map of rowops.hip),
//    32 rows per pass.
// Forward writes what the backward and the weight gradients read (r, a, mean, rstd; NULL
// pointers skip them in eval).  Backward starts from dL/da of the last layer (head.hip), writes
// dlin per layer (the weight gradients' dY) and dX of the tower input, and leaves per-workgroup
// partial column sums [dbias | dgamma | dbeta] per layer for one deferred reduction each.
//
// Device code (shared by mlp_tower.hip and the fused attention + tower kernels of tower_fused.hip):
// everything lives in namespace ncf_mlp, internal linkage per translation unit.
#pragma once
#include "ncf_common.h"

namespace ncf_mlp {
namespace {

#ifndef NCF_BWD_RING
#define NCF_BWD_RING 4
#endif
// 16-row MFMA row tiles per workgroup: 5 (80 rows: 256 workgroups = one per CU at 20,480 rows);
// tower_fused_small.hip builds the same code with 1 (the small-batch tiles)
#ifndef NCF_MLP_RT
#define NCF_MLP_RT 5
#endif
constexpr int kRT = NCF_MLP_RT;
constexpr int kRows = 16 * kRT;
constexpr int kThreads = 512;          // 8 waves
constexpr int kWaves = kThreads / 64;
constexpr int kPQ = 260;   // pitch of buffer Q (<= 256 columns)
constexpr int kPP = 132;   // pitch of buffer P (<= 128 columns; also the 8 x 3 x 256 scratch)
constexpr int N0 = 256, N1 = 128, N2 = 64;
// floats of buffer P in the backward: its rows, or the layer-0 LayerNorm backward's column-sum
// scratch (8 waves x 3 x 256) where the tile has fewer than 47 rows
constexpr int kPSize = kRows * kPP > kWaves * 3 * N0 ? kRows * kPP : kWaves * 3 * N0;
// Partial-row layout per input width K0 (= D, the embedding width: 64 or 128).
// Head partials (offsets): the flat gradient buffer's order of the head parameters, each 16-B
// aligned: mf_output.weight [K0] @0, mf_output.bias @K0, mlp_output.weight [64] @K0+4,
// mlp_output.bias @K0+68, final.0.weight [2] @K0+72, final.0.bias @K0+76; the BCE sum @K0+80
// (K0 = 64: 0, 64, 68, 132, 136, 140, 144).  Then the fused weight gradients dW0 [256 x K0] |
// dW1 [128 x 256] | dW2 [64 x 128].
template <int K0>
struct Lay {
  static constexpr int kHmfW = 0, kHmfB = K0, kHmlW = K0 + 4, kHmlB = kHmlW + N2, kHfW = kHmlB + 4,
                       kHfB = kHfW + 4, kHloss = kHfB + 4;
  static constexpr int kHeadW = kHloss + 4;
  static constexpr int kPartS = 3 * (N0 + N1 + N2) + kHeadW;   // bias/gamma/beta + head partials
  static constexpr int kW0 = kPartS, kW1 = kW0 + N0 * K0, kW2 = kW1 + N1 * N0;
  static constexpr int kPartW = kW2 + N2 * N1;   // partial floats per workgroup
};
static_assert(Lay<64>::kHeadW == 148 && Lay<64>::kPartW == 58836, "C2 partial layout");
constexpr int kPasses = (kRows * 16 + kThreads - 1) / kThreads;   // row-op passes (16 lanes/row)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Phase timestamps (diagnostic builds only, -DNCF_MLP_STAMPS; tools/mlp_stamps.py): thread 0 of
// each workgroup records the shader clock after every barrier of the tower kernels.
#ifdef NCF_MLP_STAMPS
__device__ unsigned long long g_mlp_stamps[2][1024][16];
#define NCF_STAMP(dir, k)                                                                  \
  do {                                                                                     \
    if (threadIdx.x == 0) g_mlp_stamps[dir][blockIdx.x & 1023][k] = clock64();            \
  } while (0)
#else
#define NCF_STAMP(dir, k) \
  do {                    \
  } while (0)
#endif

struct TowerArgs {
  ncf_mlp_layer l[3];
  uint64_t seed[3];
};

__device__ __forceinline__ float4 lds4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Stores of data no later phase of THIS kernel reads (weight-gradient / column-sum partials,
// the GMF row gradients): non-temporal, so the 232 KB of partials per workgroup do not evict
// the pre-LayerNorm rows r that the next phases re-read from L2.
#ifndef NCF_MLP_NT
#define NCF_MLP_NT 0   // measured: 80 -> 88 us per k_mlp_bwd with nt partials (knob kept)
#endif
__device__ __forceinline__ void st_nt(float* p, float v) {
#if NCF_MLP_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void st4_nt(float* p, float4 v) {
#if NCF_MLP_NT
  typedef float v4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(v4{v.x, v.y, v.z, v.w}, reinterpret_cast<v4*>(p));
#else
  st4(p, v);
#endif
}
__device__ __forceinline__ void lds4_st(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// LayerNorm affine of a centred float4 (x - mean) and the dropout keep-scales: ONE definition
// shared by the forward (ln_fwd) and the backward's recompute of the activation a = Dropout(LN(r))
// (act4), so both produce the same bits.
__device__ __forceinline__ float4 ln_affine(float4 xc, float rstd, float4 gg, float4 bb) {
  return make_float4(__builtin_fmaf(xc.x * rstd, gg.x, bb.x), __builtin_fmaf(xc.y * rstd, gg.y, bb.y),
                     __builtin_fmaf(xc.z * rstd, gg.z, bb.z), __builtin_fmaf(xc.w * rstd, gg.w, bb.w));
}

__device__ __forceinline__ float4 drop4(float4 y, uint64_t seed, uint64_t idx4, float p, float inv_keep) {
  if (p > 0.0f) {
    const float4 k = ncf_dropout_scale4(seed, idx4, p, inv_keep);
    y.x *= k.x; y.y *= k.y; y.z *= k.z; y.w *= k.w;
  }
  return y;
}

// a[row][col..col+3] of layer L recomputed from the saved pre-LN rows r and the row statistics
// (the forward does not store a when the backward recomputes it: 4 B/element of HBM writes and
// reads saved, r is read anyway)
template <int N>
__device__ __forceinline__ float4 act4(const ncf_mlp_layer& L, int64_t row, int col, float p,
                                       uint64_t seed, float inv_keep) {
  const float mu = L.mean[row], rs = L.rstd[row];
  const float4 x = ld4(L.r + row * N + col);
  const float4 y = ln_affine(make_float4(x.x - mu, x.y - mu, x.z - mu, x.w - mu), rs,
                             ld4(L.gamma + col), ld4(L.beta + col));
  return drop4(y, seed, ((uint64_t)row * N + col) >> 2, p, inv_keep);
}

// bf16 MFMA (the bf16 configuration, BF=true): operands rounded to bf16 (v_cvt_pk_bf16_f32),
// fp32 accumulate.  The k-permuted fp32 layout carries over unchanged: the float4 a lane group
// feeds to 4 consecutive f32 MFMA k-steps is exactly the 4-element k slot of lane group g in
// v_mfma_f32_16x16x16_bf16, and two adjacent float4 chunks are its 8-element slot in
// v_mfma_f32_16x16x32_bf16 (one instruction instead of eight f32 ones).
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16v4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x4_t pk4(float a, float b, float c, float d) {
  const bf16v4_t v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  return __builtin_bit_cast(bf16x4_t, v);
}
__device__ __forceinline__ bf16x8_t pk8(float4 a, float4 b) {
  return bf16x8_t{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                  (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
}
__device__ __forceinline__ f32x4 mfma_k32(bf16x8_t a, bf16x8_t b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}

// Split operands (MM = 3, the fp32 tower's Linears on bf16 matrix cores): every fp32 operand
// x = h + m + l, three bf16 terms each rounded to nearest (h holds x's top 8 significant bits, m
// the next 8, l the next 8: fp32's 24-bit significand; each residual is exact in fp32).  A
// product a.b is accumulated from the six bf16 x bf16 products of order >= 2^-16 (ah bh, then
// ah bm + am bh + ah bl + am bm + al bh into a second accumulator; every bf16 product is exact
// in fp32); the three dropped ones are below 2^-24 |a||b| together, the fp32 MFMA's own rounding
// level.  Six v_mfma_f32_16x16x32_bf16 (16 cycles each) replace eight v_mfma_f32_16x16x4_f32
// (32 cycles each) per 16x16x32 tile.
__device__ __forceinline__ void split3(float4 a, float4 b, bf16x8_t& h, bf16x8_t& m,
                                       bf16x8_t& l) {
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const __bf16 xh = (__bf16)x[k];
    const float r1 = x[k] - (float)xh;
    const __bf16 xm = (__bf16)r1;
    const float r2 = r1 - (float)xm;
    h[k] = xh;
    m[k] = xm;
    l[k] = (__bf16)r2;
  }
}
struct Split3 {
  bf16x8_t h, m, l;
};
__device__ __forceinline__ Split3 split3(float4 a, float4 b) {
  Split3 s;
  split3(a, b, s.h, s.m, s.l);
  return s;
}
// hi += ah bh; lo += the five cross products (see split3)
__device__ __forceinline__ void mfma_x3(const Split3& a, const Split3& b, f32x4& hi, f32x4& lo) {
  hi = mfma_k32(a.h, b.h, hi);
  lo = mfma_k32(a.h, b.m, lo);
  lo = mfma_k32(a.m, b.h, lo);
  lo = mfma_k32(a.h, b.l, lo);
  lo = mfma_k32(a.m, b.m, lo);
  lo = mfma_k32(a.l, b.h, lo);
}

__device__ __forceinline__ f32x4 mfma4(float4 a, float4 b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}

// Work split of an [80 x N] Linear output over the 8 waves: NS = N/16 column slices; with
// NS >= 8 wave w takes slices w + 8j for all 5 row tiles, with NS < 8 (N = 64) slice w % NS for
// the row tiles rt = w / NS + S r (S = 8 / NS).  A wave loads each weight chunk once and feeds
// it to all its row tiles (independent MFMA chains): 5 x reuse of every weight byte from L2.
template <int N, int RT = kRT>
struct Split {
  static constexpr int NS = N / 16;
  static constexpr int S = NS >= kWaves ? 1 : kWaves / NS;
  static constexpr int CPW = NS >= kWaves ? NS / kWaves : 1;   // column slices per wave
  static constexpr int RPW = (RT + S - 1) / S;                  // row tiles per wave (max)
  __device__ static int cs(int w, int j) { return NS >= kWaves ? w + kWaves * j : w % NS; }
  __device__ static int rt(int w, int r) { return NS >= kWaves ? r : w / NS + S * r; }
};

// Y[80 x N] = relu(X[80 x K] . W^T + b)   (W row-major [N][ldw], first K columns)
// lin_fwd on split operands (MM = 3): column slices innermost (one A split per row tile and k
// chunk), weights split as they are loaded.
template <int K, int N, int PX, int PY, int RT>
__device__ __forceinline__ void lin_fwd_x3(const float* __restrict__ X, float* __restrict__ Y,
                                           const float* __restrict__ W, int64_t ldw,
                                           const float* __restrict__ bias) {
  using Sp = Split<N, RT>;
  constexpr int KQ = K / 4, CPW = Sp::CPW, RPW = Sp::RPW;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 15, g = l >> 4;
  const float* wp[CPW];
#pragma unroll
  for (int j = 0; j < CPW; ++j) wp[j] = W + (int64_t)(16 * Sp::cs(w, j) + i) * ldw + g * KQ;
  f32x4 hi[CPW][RPW], lo[CPW][RPW];
#pragma unroll
  for (int j = 0; j < CPW; ++j)
#pragma unroll
    for (int r = 0; r < RPW; ++r) hi[j][r] = lo[j][r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < KQ / 8; ++c) {
    Split3 b[CPW];
#pragma unroll
    for (int j = 0; j < CPW; ++j) b[j] = split3(ld4(wp[j] + 8 * c), ld4(wp[j] + 8 * c + 4));
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int rt = Sp::rt(w, r);
      if (rt < RT) {
        const float* xa = X + (16 * rt + i) * PX + g * KQ + 8 * c;
        const Split3 a = split3(lds4(xa), lds4(xa + 4));
#pragma unroll
        for (int j = 0; j < CPW; ++j) mfma_x3(a, b[j], hi[j][r], lo[j][r]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < CPW; ++j) {
    const int cs = Sp::cs(w, j);
    const float bb = bias[16 * cs + i];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int rt = Sp::rt(w, r);
      if (rt < RT) {
        float* yp = Y + (16 * rt + 4 * g) * PY + 16 * cs + i;
        const f32x4 v = hi[j][r] + lo[j][r];
#pragma unroll
        for (int e = 0; e < 4; ++e) yp[e * PY] = fmaxf(v[e] + bb, 0.0f);
      }
    }
  }
}

template <int K, int N, int PX, int PY, int RT = kRT, int MM = 0>
__device__ __forceinline__ void lin_fwd(const float* __restrict__ X, float* __restrict__ Y,
                                        const float* __restrict__ W, int64_t ldw,
                                        const float* __restrict__ bias) {
  if constexpr (MM == 3) {
    lin_fwd_x3<K, N, PX, PY, RT>(X, Y, W, ldw, bias);
    return;
  }
  using Sp = Split<N, RT>;
  constexpr int KQ = K / 4;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 15, g = l >> 4;
#pragma unroll
  for (int j = 0; j < Sp::CPW; ++j) {
    const int cs = Sp::cs(w, j);
    const float* wp = W + (int64_t)(16 * cs + i) * ldw + g * KQ;
    f32x4 acc[Sp::RPW];
#pragma unroll
    for (int r = 0; r < Sp::RPW; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (MM == 1) {
#pragma unroll
      for (int c = 0; c < KQ / 8; ++c) {
        const bf16x8_t b = pk8(ld4(wp + 8 * c), ld4(wp + 8 * c + 4));
#pragma unroll
        for (int r = 0; r < Sp::RPW; ++r) {
          const int rt = Sp::rt(w, r);
          const float* xa = X + (16 * rt + i) * PX + g * KQ + 8 * c;
          if (rt < RT) acc[r] = mfma_k32(pk8(lds4(xa), lds4(xa + 4)), b, acc[r]);
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < KQ / 4; ++c) {
        const float4 b = ld4(wp + 4 * c);
#pragma unroll
        for (int r = 0; r < Sp::RPW; ++r) {
          const int rt = Sp::rt(w, r);
          if (rt < RT) acc[r] = mfma4(lds4(X + (16 * rt + i) * PX + g * KQ + 4 * c), b, acc[r]);
        }
      }
    }
    const float bb = bias[16 * cs + i];
#pragma unroll
    for (int r = 0; r < Sp::RPW; ++r) {
      const int rt = Sp::rt(w, r);
      if (rt < RT) {
        float* yp = Y + (16 * rt + 4 * g) * PY + 16 * cs + i;   // C: rows 4g + e, column 16cs + i
#pragma unroll
        for (int e = 0; e < 4; ++e) yp[e * PY] = fmaxf(acc[r][e] + bb, 0.0f);
      }
    }
  }
}

// G[80 x NO] = DL[80 x KC] . W   (W row-major [KC][ldw], first NO columns)
// lin_bwd on split operands (MM = 3): the column-slice loop innermost, so each row tile's A
// fragment (LDS) is split once per k chunk and feeds every column slice of the wave; the weight
// columns come through one ring per slice.
template <int KC, int NO, int PD, int PG>
__device__ __forceinline__ void lin_bwd_x3(const float* __restrict__ DL, float* __restrict__ G,
                                           const float* __restrict__ W, int64_t ldw) {
  using Sp = Split<NO>;
  constexpr int KQ = KC / 4, NC = KQ / 4, CPW = Sp::CPW, RPW = Sp::RPW;
  static_assert(NC % 2 == 0, "split pairs of k chunks");
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 15, g = l >> 4;
  const float* wp[CPW];
#pragma unroll
  for (int j = 0; j < CPW; ++j) wp[j] = W + (int64_t)(g * KQ) * ldw + 16 * Sp::cs(w, j) + i;
  auto chunk = [&](int j, int c) {
    const float* q = wp[j] + (int64_t)(4 * c) * ldw;
    return make_float4(q[0], q[ldw], q[2 * ldw], q[3 * ldw]);
  };
  f32x4 hi[CPW][RPW], lo[CPW][RPW];
#pragma unroll
  for (int j = 0; j < CPW; ++j)
#pragma unroll
    for (int r = 0; r < RPW; ++r) hi[j][r] = lo[j][r] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 nb[CPW][2];
#pragma unroll
  for (int j = 0; j < CPW; ++j) { nb[j][0] = chunk(j, 0); nb[j][1] = chunk(j, 1); }
#pragma unroll
  for (int c = 0; c < NC; c += 2) {
    Split3 b[CPW];
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      b[j] = split3(nb[j][0], nb[j][1]);
      if (c + 2 < NC) { nb[j][0] = chunk(j, c + 2); nb[j][1] = chunk(j, c + 3); }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int rt = Sp::rt(w, r);
      if (rt < kRT) {
        const float* da = DL + (16 * rt + i) * PD + g * KQ + 4 * c;
        const Split3 a = split3(lds4(da), lds4(da + 4));
#pragma unroll
        for (int j = 0; j < CPW; ++j) mfma_x3(a, b[j], hi[j][r], lo[j][r]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < CPW; ++j) {
    const int cs = Sp::cs(w, j);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int rt = Sp::rt(w, r);
      if (rt < kRT) {
        float* gp = G + (16 * rt + 4 * g) * PG + 16 * cs + i;
        const f32x4 v = hi[j][r] + lo[j][r];
#pragma unroll
        for (int e = 0; e < 4; ++e) gp[e * PG] = v[e];
      }
    }
  }
}

template <int KC, int NO, int PD, int PG, int MM = 0>
__device__ __forceinline__ void lin_bwd(const float* __restrict__ DL, float* __restrict__ G,
                                        const float* __restrict__ W, int64_t ldw) {
  if constexpr (MM == 3) {
    lin_bwd_x3<KC, NO, PD, PG>(DL, G, W, ldw);
    return;
  }
  using Sp = Split<NO>;
  constexpr int KQ = KC / 4;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 15, g = l >> 4;
#pragma unroll
  for (int j = 0; j < Sp::CPW; ++j) {
    const int cs = Sp::cs(w, j);
    const float* wp = W + (int64_t)(g * KQ) * ldw + 16 * cs + i;
    f32x4 acc[Sp::RPW];
#pragma unroll
    for (int r = 0; r < Sp::RPW; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    // strided weight columns: a ring of NCF_BWD_RING chunks keeps the scalar loads ahead
    constexpr int NC = KQ / 4;
    constexpr int D = NCF_BWD_RING < NC ? NCF_BWD_RING : NC;
    auto chunk = [&](int c) {
      const float* q = wp + (int64_t)(4 * c) * ldw;
      return make_float4(q[0], q[ldw], q[2 * ldw], q[3 * ldw]);
    };
    float4 ring[D];
#pragma unroll
    for (int c = 0; c < D; ++c) ring[c] = chunk(c);
    if constexpr (MM == 1) {
      static_assert(D % 2 == 0 && NC % 2 == 0, "bf16 pairs ring chunks");
#pragma unroll
      for (int c = 0; c < NC; c += 2) {
        const bf16x8_t b = pk8(ring[c % D], ring[(c + 1) % D]);
        if (c + D < NC) ring[c % D] = chunk(c + D);
        if (c + 1 + D < NC) ring[(c + 1) % D] = chunk(c + 1 + D);
#pragma unroll
        for (int r = 0; r < Sp::RPW; ++r) {
          const int rt = Sp::rt(w, r);
          const float* da = DL + (16 * rt + i) * PD + g * KQ + 4 * c;
          if (rt < kRT) acc[r] = mfma_k32(pk8(lds4(da), lds4(da + 4)), b, acc[r]);
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float4 b = ring[c % D];
        if (c + D < NC) ring[c % D] = chunk(c + D);
#pragma unroll
        for (int r = 0; r < Sp::RPW; ++r) {
          const int rt = Sp::rt(w, r);
          if (rt < kRT) acc[r] = mfma4(lds4(DL + (16 * rt + i) * PD + g * KQ + 4 * c), b, acc[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < Sp::RPW; ++r) {
      const int rt = Sp::rt(w, r);
      if (rt < kRT) {
        float* gp = G + (16 * rt + 4 * g) * PG + 16 * cs + i;
#pragma unroll
        for (int e = 0; e < 4; ++e) gp[e * PG] = acc[r][e];
      }
    }
  }
}

// LayerNorm + dropout of the ReLU rows in Y, in place (the next layer's input); saves r, a,
// mean, rstd.  16 lanes per row, kPasses passes over the 80 rows.  With hw != NULL, also the
// head: mlp_pred = a . hw + b_out, prob = sigmoid(w0 mf_pred + w1 mlp_pred + b_fin).
template <int N, int PY, int RT = kRT>
__device__ __forceinline__ void ln_fwd(float* __restrict__ Y, int64_t row0, int rows,
                                       const ncf_mlp_layer& L, float eps, float p, uint64_t seed,
                                       const float* __restrict__ hw, const float* __restrict__ b_out,
                                       const float* __restrict__ mf_pred,
                                       const float* __restrict__ w_fin,
                                       const float* __restrict__ b_fin,
                                       float* __restrict__ mlp_pred, float* __restrict__ prob) {
  // The kPasses row passes of a lane run interleaved (independent chains: the shuffle
  // reductions of one pass hide behind the arithmetic of the others).  A pass whose row is past
  // the tile (rr >= kRows: waves 4-7 in the last pass) computes on zeros and stores nothing.
  // No fp contraction here: the unrolled passes must round identically, so a row's result does
  // not depend on which pass (= its position in the tile, i.e. the batch) computes it; the
  // fused multiply-adds are explicit.
#pragma clang fp contract(off)
  constexpr int CH = N / 64, TR = 16 * RT, NP = (TR * 16 + kThreads - 1) / kThreads;
  const int sub = threadIdx.x & 15;
  const float inv_keep = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  float4 x[NP][CH];
  float s[NP], mean[NP], rstd[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int rr = (threadIdx.x >> 4) + q * (kThreads / 16);
    s[q] = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 16 + sub) * 4;
      x[q][c] = rr < TR ? lds4(Y + rr * PY + col) : make_float4(0.f, 0.f, 0.f, 0.f);
      s[q] += x[q][c].x + x[q][c].y + x[q][c].z + x[q][c].w;
    }
  }
  if (L.r) {
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int rr = (threadIdx.x >> 4) + q * (kThreads / 16);
      if (rr < rows) {
#pragma unroll
        for (int c = 0; c < CH; ++c) st4(L.r + (row0 + rr) * N + (c * 16 + sub) * 4, x[q][c]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) mean[q] = group_sum<16>(s[q]) * (1.0f / N);
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    s[q] = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      float4& v = x[q][c];
      v.x -= mean[q]; v.y -= mean[q]; v.z -= mean[q]; v.w -= mean[q];
      s[q] = __builtin_fmaf(v.x, v.x, s[q]); s[q] = __builtin_fmaf(v.y, v.y, s[q]);
      s[q] = __builtin_fmaf(v.z, v.z, s[q]); s[q] = __builtin_fmaf(v.w, v.w, s[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) rstd[q] = 1.0f / sqrtf(group_sum<16>(s[q]) * (1.0f / N) + eps);
  float dot[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int rr = (threadIdx.x >> 4) + q * (kThreads / 16);
    const int64_t row = row0 + rr;
    const bool ok = rr < rows;
    dot[q] = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 16 + sub) * 4;
      const float4 y = drop4(ln_affine(x[q][c], rstd[q], ld4(L.gamma + col), ld4(L.beta + col)),
                             seed, ((uint64_t)row * N + col) >> 2, p, inv_keep);
      if (rr < TR) lds4_st(Y + rr * PY + col, y);
      if (ok && L.a) st4(L.a + row * N + col, y);
      if (hw) {
        const float4 h = ld4(hw + col);
        dot[q] = fmaf(y.x, h.x, dot[q]); dot[q] = fmaf(y.y, h.y, dot[q]);
        dot[q] = fmaf(y.z, h.z, dot[q]); dot[q] = fmaf(y.w, h.w, dot[q]);
      }
    }
    if (ok && sub == 0 && L.mean) {
      L.mean[row] = mean[q];
      L.rstd[row] = rstd[q];
    }
  }
  if (hw) {
#pragma unroll
    for (int q = 0; q < NP; ++q) dot[q] = group_sum<16>(dot[q]);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int rr = (threadIdx.x >> 4) + q * (kThreads / 16);
      const int64_t row = row0 + rr;
      if (rr < rows && sub == 0) {
        const float mp = dot[q] + b_out[0];
        mlp_pred[row] = mp;
        const float z = w_fin[0] * mf_pred[row] + w_fin[1] * mp + b_fin[0];
        prob[row] = 1.0f / (1.0f + expf(-z));
      }
    }
  }
}

// Backward of dropout -> LayerNorm -> ReLU for the 80 rows, in place: G (dL/da) -> dL/dlin
// (also to HBM); this workgroup's column sums [dbias | dgamma | dbeta] -> part[0 : 3N), through
// the free buffer S (8 waves x 3N floats).
// R: the layer's pre-LN rows r staged in LDS by stage_act (pitch kPQ, mean / rstd at columns
// N, N + 1), or NULL to read them from HBM; S may overlap R (a barrier separates them).
template <int N, int PG>
__device__ __forceinline__ void ln_bwd(float* __restrict__ G, float* __restrict__ S, int64_t row0,
                                       int rows, const ncf_mlp_layer& L, float p, uint64_t seed,
                                       float* __restrict__ part, const float* R = nullptr) {
  constexpr int CH = N / 64;
  const int sub = threadIdx.x & 15;
  const int wv = threadIdx.x >> 6;
  const float inv_keep = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  float4 sl[CH], sg[CH], sb[CH];   // this lane's column sums over its rows
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    sl[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    sg[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    sb[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int pass = 0; pass < kPasses; ++pass) {
    const int rr = (threadIdx.x >> 4) + pass * (kThreads / 16);
    if (rr >= kRows) break;
    const int64_t row = row0 + rr;
    const bool ok = rr < rows;
    const float mu = ok ? (R ? R[rr * kPQ + N] : L.mean[row]) : 0.0f;
    const float rs = ok ? (R ? R[rr * kPQ + N + 1] : L.rstd[row]) : 0.0f;
    float4 gd[CH], xh[CH];
    uint32_t pos = 0;   // ReLU mask: bit 4c + e <=> r > 0
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 16 + sub) * 4;
      float4 d = lds4(G + rr * PG + col);
      if (p > 0.0f) {
        const float4 k = ncf_dropout_scale4(seed, ((uint64_t)row * N + col) >> 2, p, inv_keep);
        d.x *= k.x; d.y *= k.y; d.z *= k.z; d.w *= k.w;
      }
      const float4 x = !ok ? make_float4(0.f, 0.f, 0.f, 0.f)
                           : R ? lds4(R + rr * kPQ + col) : ld4(L.r + row * N + col);
      const float4 gg = ld4(L.gamma + col);
      const float4 h = make_float4((x.x - mu) * rs, (x.y - mu) * rs, (x.z - mu) * rs, (x.w - mu) * rs);
      pos |= ((x.x > 0.0f ? 1u : 0u) | (x.y > 0.0f ? 2u : 0u) | (x.z > 0.0f ? 4u : 0u) |
              (x.w > 0.0f ? 8u : 0u)) << (4 * c);
      sg[c].x += d.x * h.x; sg[c].y += d.y * h.y; sg[c].z += d.z * h.z; sg[c].w += d.w * h.w;
      sb[c].x += d.x; sb[c].y += d.y; sb[c].z += d.z; sb[c].w += d.w;
      gd[c] = make_float4(d.x * gg.x, d.y * gg.y, d.z * gg.z, d.w * gg.w);
      s1 += gd[c].x + gd[c].y + gd[c].z + gd[c].w;
      s2 += gd[c].x * h.x + gd[c].y * h.y + gd[c].z * h.z + gd[c].w * h.w;
      xh[c] = h;
    }
    const float m1 = group_sum<16>(s1) * (1.0f / N);
    const float m2 = group_sum<16>(s2) * (1.0f / N);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 16 + sub) * 4;
      const uint32_t mk = pos >> (4 * c);
      float4 o;
      o.x = (mk & 1u) ? rs * (gd[c].x - m1 - xh[c].x * m2) : 0.0f;
      o.y = (mk & 2u) ? rs * (gd[c].y - m1 - xh[c].y * m2) : 0.0f;
      o.z = (mk & 4u) ? rs * (gd[c].z - m1 - xh[c].z * m2) : 0.0f;
      o.w = (mk & 8u) ? rs * (gd[c].w - m1 - xh[c].w * m2) : 0.0f;
      lds4_st(G + rr * PG + col, o);
      if (ok && L.dlin) st4(L.dlin + row * N + col, o);
      sl[c].x += o.x; sl[c].y += o.y; sl[c].z += o.z; sl[c].w += o.w;
    }
  }
  // over the 4 row groups of the wave (lanes sub, sub + 16, sub + 32, sub + 48), then the waves
#define NCF_R4(v)                                  \
  v += __shfl_xor(v, 16, 64);                      \
  v += __shfl_xor(v, 32, 64);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    NCF_R4(sl[c].x) NCF_R4(sl[c].y) NCF_R4(sl[c].z) NCF_R4(sl[c].w)
    NCF_R4(sg[c].x) NCF_R4(sg[c].y) NCF_R4(sg[c].z) NCF_R4(sg[c].w)
    NCF_R4(sb[c].x) NCF_R4(sb[c].y) NCF_R4(sb[c].z) NCF_R4(sb[c].w)
  }
#undef NCF_R4
  if (R) __syncthreads();   // every wave's reads of the stash are done before S overwrites it
  if ((threadIdx.x & 63) < 16) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 16 + sub) * 4;
      lds4_st(S + wv * 3 * N + col, sl[c]);
      lds4_st(S + wv * 3 * N + N + col, sg[c]);
      lds4_st(S + wv * 3 * N + 2 * N + col, sb[c]);
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 3 * N; e += kThreads) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += S[w * 3 * N + e];
    st_nt(part + e, s);
  }
  __syncthreads();
}

// The forward in workgroups of VR valid rows staged as RT 16-row MFMA tiles (the padding rows
// are zeros and are never stored).  VR < 16 RT lets two workgroups share a CU (A/B knob).
// x_staged: the caller has put the input rows (zeros past the batch) into buffer P already (the
// attention block fused ahead of the tower, tower_fused.hip)
template <int K0, int RT, int VR, int MM = 0>
__device__ __forceinline__ void mlp_fwd_body(float* __restrict__ lds,
    const float* __restrict__ xin, int64_t n, TowerArgs a, float eps, float p,
    const ncf_step_clock* clock, const float* __restrict__ w_out, const float* __restrict__ b_out,
    const float* __restrict__ mf_pred, const float* __restrict__ w_fin,
    const float* __restrict__ b_fin, float* __restrict__ mlp_pred, float* __restrict__ prob, bool x_staged) {
  constexpr int TR = 16 * RT;
  float* Q = lds;                  // [TR][kPQ]: layer 0 out (256), layer 2 out (64)
  float* P = lds + TR * kPQ;       // [TR][kPP]: input x (64), layer 1 out (128)
  const int64_t row0 = (int64_t)blockIdx.x * VR;
  const int rows = (int)min<int64_t>(VR, n - row0);
  const uint64_t cs = clock ? clock->seed : 0ull;
  NCF_STAMP(0, 0);
  if (!x_staged) {   // the input rows, every load in flight before the first LDS store
    constexpr int TOT = TR * (K0 / 4), IT = (TOT + kThreads - 1) / kThreads;
    float4 v[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      const int e = threadIdx.x + kThreads * j, r = e / (K0 / 4), c = (e % (K0 / 4)) * 4;
      v[j] = (e < TOT && r < rows) ? ld4(xin + (row0 + r) * K0 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      const int e = threadIdx.x + kThreads * j, r = e / (K0 / 4), c = (e % (K0 / 4)) * 4;
      if (e < TOT) lds4_st(P + r * kPP + c, v[j]);
    }
  }
  __syncthreads();
  NCF_STAMP(0, 1);
  lin_fwd<K0, N0, kPP, kPQ, RT, MM>(P, Q, a.l[0].w, a.l[0].ldw, a.l[0].b);
  __syncthreads();
  NCF_STAMP(0, 2);
  ln_fwd<N0, kPQ, RT>(Q, row0, rows, a.l[0], eps, p, a.seed[0] + cs, nullptr, nullptr, nullptr,
                      nullptr, nullptr, nullptr, nullptr);
  __syncthreads();
  NCF_STAMP(0, 3);
  lin_fwd<N0, N1, kPQ, kPP, RT, (MM == 3 ? 0 : MM)>(Q, P, a.l[1].w, a.l[1].ldw, a.l[1].b);
  __syncthreads();
  NCF_STAMP(0, 4);
  ln_fwd<N1, kPP, RT>(P, row0, rows, a.l[1], eps, p, a.seed[1] + cs, nullptr, nullptr, nullptr,
                      nullptr, nullptr, nullptr, nullptr);
  __syncthreads();
  NCF_STAMP(0, 5);
  lin_fwd<N1, N2, kPP, kPQ, RT, MM>(P, Q, a.l[2].w, a.l[2].ldw, a.l[2].b);
  __syncthreads();
  NCF_STAMP(0, 6);
  ln_fwd<N2, kPQ, RT>(Q, row0, rows, a.l[2], eps, p, a.seed[2] + cs, w_out, b_out, mf_pred, w_fin,
                      b_fin, mlp_pred, prob);
#ifdef NCF_MLP_STAMPS
  __syncthreads();
#endif
  NCF_STAMP(0, 7);
}

template <int K0, int RT, int VR, int MM = 0>
__global__ __launch_bounds__(kThreads) void k_mlp_fwd(
    const float* __restrict__ xin, int64_t n, TowerArgs a, float eps, float p,
    const ncf_step_clock* clock, const float* __restrict__ w_out, const float* __restrict__ b_out,
    const float* __restrict__ mf_pred, const float* __restrict__ w_fin,
    const float* __restrict__ b_fin, float* __restrict__ mlp_pred, float* __restrict__ prob) {
  extern __shared__ float lds[];
  mlp_fwd_body<K0, RT, VR, MM>(lds, xin, n, a, eps, p, clock, w_out, b_out, mf_pred, w_fin, b_fin,
                               mlp_pred, prob, false);
}

#ifndef NCF_FWD_RT
#define NCF_FWD_RT 5
#endif
#ifndef NCF_FWD_VR
#define NCF_FWD_VR 80
#endif
constexpr int kFwdRT = NCF_FWD_RT, kFwdVR = NCF_FWD_VR;
static_assert(kFwdVR <= 16 * kFwdRT, "forward rows per workgroup exceed its tiles");

// Weight gradient of one Linear over this workgroup's 80 rows: out[n][k] = sum_r dlin[r][n] X[r][k]
// (the partial of this workgroup; one deferred reduction sums the 256 partial rows).  16x16
// output tiles, contraction over the rows k-permuted: lane group g covers rows [20g, 20g + 20).
// A wave keeps its dlin column fragment (20 values) and sweeps its k tiles with it.
template <int N, int K, int PG, int PX, int MM = 0>
__device__ __forceinline__ void wgrad_layer(const float* __restrict__ G, const float* __restrict__ X,
                                            float* __restrict__ out) {
  static_assert(MM == 0 || MM == 1, "weight gradients: fp32 or single-term bf16 MFMA");
  constexpr bool BF = MM == 1;
  constexpr int TN = N / 16, TK = K / 16, R4 = kRows / 4;
  constexpr int TNW = TN >= kWaves ? TN / kWaves : 1;        // n tiles per wave
  constexpr int WPN = TN >= kWaves ? 1 : kWaves / TN;        // waves per n tile
  constexpr int TKW = TK / WPN;                              // k tiles per wave
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 15, g = l >> 4;
#pragma unroll
  for (int jn = 0; jn < TNW; ++jn) {
    const int tn = TN >= kWaves ? w + kWaves * jn : w % TN;
    const int tk0 = TN >= kWaves ? 0 : (w / TN) * TKW;
    float af[R4];
#pragma unroll
    for (int s = 0; s < R4; ++s) af[s] = G[(g * R4 + s) * PG + 16 * tn + i];
#pragma unroll 2
    for (int jk = 0; jk < TKW; ++jk) {
      const int tk = tk0 + jk;
      const float* xb = X + (g * R4) * PX + 16 * tk + i;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {     // 4 consecutive rows of the contraction per 16x16x16 bf16 MFMA
        static_assert(R4 % 4 == 0, "rows per lane group");
#pragma unroll
        for (int s = 0; s < R4; s += 4) {
          const bf16x4_t a4 = pk4(af[s], af[s + 1], af[s + 2], af[s + 3]);
          const bf16x4_t b4 = pk4(xb[s * PX], xb[(s + 1) * PX], xb[(s + 2) * PX], xb[(s + 3) * PX]);
          if ((s / 4) & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc1, 0, 0, 0);
          else acc0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc0, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int s = 0; s < R4; s += 2) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], xb[s * PX], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s + 1], xb[(s + 1) * PX], acc1, 0, 0, 0);
        }
      }
      float* o = out + (16 * tn + 4 * g) * K + 16 * tk + i;
#pragma unroll
      for (int e = 0; e < 4; ++e) st_nt(o + e * K, acc0[e] + acc1[e]);
    }
  }
}

// the activation rows a of layer L into LDS: loaded when the forward saved them, else
// recomputed from r (act4's arithmetic: the same bits).  NCF_STAGE_BATCH = SB iterations' loads
// issued before their uses (measured at C2, ms/step: SB 1 0.3075, 5 0.3100, 10 0.3087 — within
// noise; the load-then-store loop's latency overlaps the other waves' work), default 1.
// (Keeping layer 1's r rows in Q's free columns from this staging to its LayerNorm backward —
// the R argument below — measured in-step, 4 interleaved runs: k_mlp_bwd 90.3 us without, 92.4
// us with (the staging loop's extra LDS stores and the barrier before the column-sum scratch);
// the tower passes R = NULL.)
#ifndef NCF_STAGE_BATCH
#define NCF_STAGE_BATCH 1
#endif
// R (recompute only, L.a == NULL): also keep the loaded r rows and their mean / rstd in LDS
// (pitch kPQ, statistics at columns K, K + 1) for the layer's LayerNorm backward.
template <int K, int PX>
__device__ __forceinline__ void stage_act(float* __restrict__ X, const ncf_mlp_layer& L,
                                          int64_t row0, int rows, float p, uint64_t seed,
                                          float* __restrict__ R = nullptr) {
  constexpr int TOT = kRows * (K / 4), IT = (TOT + kThreads - 1) / kThreads;
  constexpr int SB = NCF_STAGE_BATCH < IT ? NCF_STAGE_BATCH : IT;
  const float inv_keep = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  for (int b0 = 0; b0 < IT; b0 += SB) {
    float4 x[SB];
    float mu[SB], rs[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int e = threadIdx.x + kThreads * (b0 + j), r = e / (K / 4), c = (e % (K / 4)) * 4;
      x[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      mu[j] = 0.0f;
      rs[j] = 0.0f;
      if (b0 + j < IT && e < TOT && r < rows) {
        const int64_t row = row0 + r;
        if (L.a) {
          x[j] = ld4(L.a + row * K + c);
        } else {
          x[j] = ld4(L.r + row * K + c);
          mu[j] = L.mean[row];
          rs[j] = L.rstd[row];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int e = threadIdx.x + kThreads * (b0 + j), r = e / (K / 4), c = (e % (K / 4)) * 4;
      if (b0 + j < IT && e < TOT) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < rows) {
          if (L.a) {
            v = x[j];
          } else {   // act4 on the loaded row values
            const float4 xx = x[j];
            const float m = mu[j];
            const float4 y = ln_affine(make_float4(xx.x - m, xx.y - m, xx.z - m, xx.w - m), rs[j],
                                       ld4(L.gamma + c), ld4(L.beta + c));
            v = drop4(y, seed, ((uint64_t)(row0 + r) * K + c) >> 2, p, inv_keep);
          }
        }
        lds4_st(X + r * PX + c, v);
        if (R) {
          lds4_st(R + r * kPQ + c, x[j]);
          if (c == 0) {
            R[r * kPQ + K] = mu[j];
            R[r * kPQ + K + 1] = rs[j];
          }
        }
      }
    }
  }
}

template <int K, int PX>
__device__ __forceinline__ void stage_rows(float* __restrict__ X, const float* __restrict__ src,
                                           int64_t row0, int rows) {
  constexpr int TOT = kRows * (K / 4), IT = (TOT + kThreads - 1) / kThreads;
  float4 v[IT];   // every load in flight before the first store
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int e = threadIdx.x + kThreads * j, r = e / (K / 4), c = (e % (K / 4)) * 4;
    v[j] = (e < TOT && r < rows) ? ld4(src + (row0 + r) * K + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int e = threadIdx.x + kThreads * j, r = e / (K / 4), c = (e % (K / 4)) * 4;
    if (e < TOT) lds4_st(X + r * PX + c, v[j]);
  }
}

// Head backward (head.hip's k_head_bwd math) for the 80 rows: dL/da_2 -> G, dL/d(LN'd GMF
// rows) -> HBM, this workgroup's head parameter partials + BCE sum -> part[0 : kHeadW) (through
// the free buffer S).  16 lanes per row, 4 columns per lane (W3 = 64) and K0/64 float4 chunks
// of the GMF rows (D = K0).
template <int K0>
__device__ __forceinline__ void head_bwd(float* __restrict__ G, float* __restrict__ S,
                                         int64_t row0, int rows, const ncf_head_args& h,
                                         const ncf_mlp_layer& L2, float p, uint64_t seed,
                                         float inv_n, float* __restrict__ part) {
  using T = Lay<K0>;
  constexpr int CM = K0 / 64;   // float4 chunks of a GMF row per lane
  const float inv_keep = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int sub = threadIdx.x & 15, wv = threadIdx.x >> 6, col = sub * 4;
  const float wf0 = h.final_w[0], wf1 = h.final_w[1];
  const float4 wo = ld4(h.mlp_out_w + col);
  float4 wm[CM], am[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    wm[c] = ld4(h.mf_out_w + 64 * c + col);
    am[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 aw = make_float4(0.f, 0.f, 0.f, 0.f);
  float sw0 = 0.f, sw1 = 0.f, sbf = 0.f, sbo = 0.f, sbm = 0.f, sl = 0.f;
  // Every pass's loads first (all of this thread's rows in flight), then the math: a
  // load-then-use loop waits one HBM latency per pass (the phase was 16.8K of the backward's
  // 192K cycles per workgroup).  Same values, same arithmetic (act4's) as loading in the loop.
  float ld_o[kPasses], ld_t[kPasses], ld_mu[kPasses], ld_rs[kPasses];
  float4 ld_x[kPasses], ld_u[kPasses][CM], ld_it[kPasses][CM];
  const float4 g2 = L2.a ? make_float4(0.f, 0.f, 0.f, 0.f) : ld4(L2.gamma + col);
  const float4 b2 = L2.a ? make_float4(0.f, 0.f, 0.f, 0.f) : ld4(L2.beta + col);
#pragma unroll
  for (int pass = 0; pass < kPasses; ++pass) {
    const int rr = (threadIdx.x >> 4) + pass * (kThreads / 16);
    const int64_t row = row0 + rr;
    if (rr < kRows && rr < rows) {
      ld_o[pass] = h.prob[row];
      ld_t[pass] = h.targets ? h.targets[row] : h.grad_prob[row];
      if (L2.a) {
        ld_x[pass] = ld4(L2.a + row * N2 + col);
      } else {
        ld_mu[pass] = L2.mean[row];
        ld_rs[pass] = L2.rstd[row];
        ld_x[pass] = ld4(L2.r + row * N2 + col);
      }
      int64_t urow = row;   // (the gather's source row of this row's LN'd user row)
      if (h.user_ids && h.group_rows > 1) {
        const int64_t f = row - row % h.group_rows;
        if (row != f && h.user_ids[row] == h.user_ids[f]) urow = f;
      }
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        const int64_t o = row * K0 + 64 * c + col;
        ld_u[pass][c] = ld4(h.mf_user_ln + urow * K0 + 64 * c + col);
        ld_it[pass][c] = ld4(h.mf_item_ln + o);
      }
    }
  }
#pragma unroll
  for (int pass = 0; pass < kPasses; ++pass) {
    const int rr = (threadIdx.x >> 4) + pass * (kThreads / 16);
    if (rr >= kRows) break;
    const int64_t row = row0 + rr;
    const bool ok = rr < rows;
    float dz = 0.f, l = 0.f;
    if (ok) {
      const float o = ld_o[pass];
      float go;
      if (h.targets) {
        const float t = ld_t[pass];
        go = inv_n * (o - t) / fmaxf((1.0f - o) * o, 1e-12f);
        if (sub == 0)   // (the BCE term: one lane of the row sums it)
          l = -(t * fmaxf(logf(o), -100.0f) + (1.0f - t) * fmaxf(logf(1.0f - o), -100.0f));
      } else {
        go = ld_t[pass];
      }
      dz = go * (1.0f - o) * o;
    }
    const float dmf = dz * wf0, dml = dz * wf1;
    lds4_st(G + rr * kPQ + col, make_float4(dml * wo.x, dml * wo.y, dml * wo.z, dml * wo.w));
    if (ok) {
      float4 x = ld_x[pass];
      if (!L2.a) {   // act4 on the loaded row values
        const float mu = ld_mu[pass], rs = ld_rs[pass];
        const float4 y = ln_affine(make_float4(x.x - mu, x.y - mu, x.z - mu, x.w - mu), rs, g2, b2);
        x = drop4(y, seed, ((uint64_t)row * N2 + col) >> 2, p, inv_keep);
      }
      aw.x += dml * x.x; aw.y += dml * x.y; aw.z += dml * x.z; aw.w += dml * x.w;
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        const int64_t o = row * K0 + 64 * c + col;
        const float4 u = ld_u[pass][c], it = ld_it[pass][c];
        const float4 gv = make_float4(dmf * wm[c].x, dmf * wm[c].y, dmf * wm[c].z, dmf * wm[c].w);
        st4_nt(h.grad_mf_user_ln + o, make_float4(gv.x * it.x, gv.y * it.y, gv.z * it.z, gv.w * it.w));
        st4_nt(h.grad_mf_item_ln + o, make_float4(gv.x * u.x, gv.y * u.y, gv.z * u.z, gv.w * u.w));
        am[c].x += dmf * u.x * it.x; am[c].y += dmf * u.y * it.y;
        am[c].z += dmf * u.z * it.z; am[c].w += dmf * u.w * it.w;
      }
      if (sub == 0) {
        sw0 += dz * h.mf_pred[row];
        sw1 += dz * h.mlp_pred[row];
        sbf += dz;
        sbo += dml;
        sbm += dmf;
        sl += l;
      }
    }
  }
#define NCF_R4(v)                                  \
  v += __shfl_xor(v, 16, 64);                      \
  v += __shfl_xor(v, 32, 64);
  NCF_R4(aw.x) NCF_R4(aw.y) NCF_R4(aw.z) NCF_R4(aw.w)
#pragma unroll
  for (int c = 0; c < CM; ++c) { NCF_R4(am[c].x) NCF_R4(am[c].y) NCF_R4(am[c].z) NCF_R4(am[c].w) }
  NCF_R4(sw0) NCF_R4(sw1) NCF_R4(sbf) NCF_R4(sbo) NCF_R4(sbm) NCF_R4(sl)
#undef NCF_R4
  float* sw = S + wv * T::kHeadW;
  if ((threadIdx.x & 63) < 16) {
#pragma unroll
    for (int c = 0; c < CM; ++c) lds4_st(sw + T::kHmfW + 64 * c + col, am[c]);
    lds4_st(sw + T::kHmlW + col, aw);
    if (sub == 0) {
      lds4_st(sw + T::kHmfB, make_float4(sbm, 0.f, 0.f, 0.f));
      lds4_st(sw + T::kHmlB, make_float4(sbo, 0.f, 0.f, 0.f));
      lds4_st(sw + T::kHfW, make_float4(sw0, sw1, 0.f, 0.f));
      lds4_st(sw + T::kHfB, make_float4(sbf, 0.f, 0.f, 0.f));
      lds4_st(sw + T::kHloss, make_float4(sl, 0.f, 0.f, 0.f));
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T::kHeadW; e += kThreads) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) v += S[w * T::kHeadW + e];
    st_nt(part + e, v);
  }
  __syncthreads();
}

// dx == NULL: the input gradient stays in buffer P (rows x K0, pitch kPP) for a consumer fused
// behind this body (the attention backward, tower_fused.hip)
// VR: the workgroup's rows (<= kRows: a tile of whole attention groups, tower_fused.hip)
template <int K0, int MM = 0, int VR = kRows>
__device__ __forceinline__ void mlp_bwd_body(float* __restrict__ lds, const float* __restrict__ g_last, int64_t n,
                                                      TowerArgs a, float p,
                                                      const ncf_step_clock* clock,
                                                      float* __restrict__ dx,
                                                      float* __restrict__ part, ncf_head_args h,
                                                      int fused_head, float inv_n,
                                                      const float* __restrict__ xin, int fused_wgrad) {
  static_assert(VR <= kRows, "rows per workgroup exceed the tile");
  float* Q = lds;
  float* P = lds + kRows * kPQ;
  const int64_t row0 = (int64_t)blockIdx.x * VR;
  const int rows = (int)min<int64_t>(VR, n - row0);
  const uint64_t cs = clock ? clock->seed : 0ull;
  using T = Lay<K0>;
  // MM = 3: the three dX Linears on split operands; the weight gradients stay on fp32 MFMA
  // (their activation operand would be split once per (n, k) tile: VALU-bound, measured slower,
  // round 5: wgrad1 29.3K vs 26.9K cycles, lin1 bwd 21.8K vs 30.8K)
  constexpr int WM = MM == 3 ? 0 : MM;
  float* pp = part + (int64_t)blockIdx.x * T::kPartW;
  NCF_STAMP(1, 0);
  if (fused_head) {
    head_bwd<K0>(Q, P, row0, rows, h, a.l[2], p, a.seed[2] + cs, inv_n, pp + 3 * (N0 + N1 + N2));
  } else {
    for (int e = threadIdx.x; e < kRows * (N2 / 4); e += kThreads) {
      const int r = e / (N2 / 4), c = (e % (N2 / 4)) * 4;
      lds4_st(Q + r * kPQ + c,
              r < rows ? ld4(g_last + (row0 + r) * N2 + c) : make_float4(0.f, 0.f, 0.f, 0.f));
    }
    __syncthreads();
  }
  NCF_STAMP(1, 1);
  ln_bwd<N2, kPQ>(Q, P, row0, rows, a.l[2], p, a.seed[2] + cs, pp);
  NCF_STAMP(1, 2);
  // r1 kept in Q's columns 128..257 (free until stage a0; dlin2 uses columns 0..63) from the
  // a1 staging to the LayerNorm backward of layer 1: one HBM read of r1 instead of two
  float* R1 = nullptr;   // (the r1 stash: see stage_act)
  if (fused_wgrad) {   // dW2 = dlin2^T a1 (a1 staged in P, then overwritten by dX)
    stage_act<N1, kPP>(P, a.l[1], row0, rows, p, a.seed[1] + cs, R1);
    __syncthreads();
    NCF_STAMP(1, 3);
    wgrad_layer<N2, N1, kPQ, kPP, WM>(Q, P, pp + T::kW2);
    __syncthreads();
    NCF_STAMP(1, 4);
  }
  lin_bwd<N2, N1, kPQ, kPP, MM>(Q, P, a.l[2].w, a.l[2].ldw);
  __syncthreads();
  NCF_STAMP(1, 5);
  ln_bwd<N1, kPP>(P, Q, row0, rows, a.l[1], p, a.seed[1] + cs, pp + 3 * N2, R1);
  NCF_STAMP(1, 6);
  if (fused_wgrad) {   // dW1 = dlin1^T a0
    stage_act<N0, kPQ>(Q, a.l[0], row0, rows, p, a.seed[0] + cs);
    __syncthreads();
    NCF_STAMP(1, 7);
    wgrad_layer<N1, N0, kPP, kPQ, WM>(P, Q, pp + T::kW1);
    __syncthreads();
    NCF_STAMP(1, 8);
  }
  lin_bwd<N1, N0, kPP, kPQ, MM>(P, Q, a.l[1].w, a.l[1].ldw);
  __syncthreads();
  NCF_STAMP(1, 9);
  ln_bwd<N0, kPQ>(Q, P, row0, rows, a.l[0], p, a.seed[0] + cs, pp + 3 * (N2 + N1));
  NCF_STAMP(1, 10);
  if (fused_wgrad) {   // dW0 = dlin0^T x (the first 64 input columns of mlp.0)
    stage_rows<K0, kPP>(P, xin, row0, rows);
    __syncthreads();
    NCF_STAMP(1, 11);
    wgrad_layer<N0, K0, kPQ, kPP, WM>(Q, P, pp + T::kW0);
    __syncthreads();
    NCF_STAMP(1, 12);
  }
  lin_bwd<N0, K0, kPQ, kPP, MM>(Q, P, a.l[0].w, a.l[0].ldw);
  __syncthreads();
  NCF_STAMP(1, 13);
  if (dx) {
    for (int e = threadIdx.x; e < rows * (K0 / 4); e += kThreads) {
      const int r = e / (K0 / 4), c = (e % (K0 / 4)) * 4;
      st4(dx + (row0 + r) * K0 + c, lds4(P + r * kPP + c));
    }
  }
#ifdef NCF_MLP_STAMPS
  __syncthreads();
#endif
  NCF_STAMP(1, 14);
}

template <int K0, int MM = 0>
__global__ __launch_bounds__(kThreads) void k_mlp_bwd(const float* __restrict__ g_last, int64_t n,
                                                      TowerArgs a, float p,
                                                      const ncf_step_clock* clock,
                                                      float* __restrict__ dx,
                                                      float* __restrict__ part, ncf_head_args h,
                                                      int fused_head, float inv_n,
                                                      const float* __restrict__ xin, int fused_wgrad) {
  extern __shared__ float lds[];
  mlp_bwd_body<K0, MM>(lds, g_last, n, a, p, clock, dx, part, h, fused_head, inv_n, xin,
                       fused_wgrad);
}

constexpr size_t kLds = sizeof(float) * (kRows * kPQ + kPSize);
constexpr size_t kLdsFwd = sizeof(float) * 16 * kFwdRT * (kPQ + kPP);
static_assert(kWaves * 3 * N0 <= kPSize, "ln_bwd scratch must fit in buffer P");
static_assert(kWaves * Lay<128>::kHeadW <= kPSize, "head scratch must fit in buffer P");
static_assert(kWaves * 3 * N1 <= kRows * kPQ, "ln_bwd scratch of layer 1 must fit in buffer Q");
static_assert(128 <= kPP - 4, "a 128-wide input fits buffer P");

bool tower_ok(int64_t dim, int64_t n_layers, const int64_t* hidden) {
  return (dim == 64 || dim == 128) && n_layers == 3 && hidden && hidden[0] == N0 &&
         hidden[1] == N1 && hidden[2] == N2;
}

int make_args(const ncf_mlp_layer* layers, uint64_t seed, int64_t dim, TowerArgs& a) {
  for (int l = 0; l < 3; ++l) {
    a.l[l] = layers[l];
    if (!a.l[l].w || !a.l[l].b || !a.l[l].gamma || !a.l[l].beta || a.l[l].ldw < (l ? 0 : dim) ||
        (a.l[l].ldw & 3)) {
      ncf_set_error("ncf_mlp: layer %d needs w/b/gamma/beta and a float4-aligned ldw", l);
      return NCF_ERR_ARG;
    }
    a.seed[l] = (seed + 0x9E37ull * (uint64_t)(l + 1)) & 0x7FFFFFFFFFFFFFFFull;
  }
  return NCF_OK;
}

// the tower backward's per-workgroup partial rows -> deferred reductions into the flat gradient
// buffer (host side; shared by mlp_tower.hip and tower_fused.hip)
template <int K0>
int defer_tower(const TowerArgs& a, const ncf_head_args* head, const ncf_head_args& h,
                       float inv_n, bool fw, int nb, float* workspace, ncf_reduce_list* lst) {
  using T = Lay<K0>;
  constexpr int PW = T::kPartW;
  int rc = NCF_OK;
  // per layer: [dbias | dgamma | dbeta] partial columns -> one strided reduction when the three
  // outputs are equally spaced (consecutive parameters of the flat gradient buffer)
  const int widths[3] = {N0, N1, N2};
  const int64_t offs[3] = {3 * (N2 + N1), 3 * N2, 0};
  for (int l = 0; l < 3 && !rc; ++l) {
    const int W = widths[l];
    const float* pp = workspace + offs[l];
    const ncf_mlp_layer& L = a.l[l];
    const ptrdiff_t s1 = L.dgamma - L.dbias, s2 = L.dbeta - L.dgamma;
    if (s1 == s2 && s1 >= W) {
      rc = ncf_defer(lst, pp, nb, PW, 3 * W, L.dbias, 0, W, s1);
    } else {
      rc = ncf_defer(lst, pp, nb, PW, W, L.dbias, 0, W, W);
      if (!rc) rc = ncf_defer(lst, pp + W, nb, PW, W, L.dgamma, 0, W, W);
      if (!rc) rc = ncf_defer(lst, pp + 2 * W, nb, PW, W, L.dbeta, 0, W, W);
    }
  }
  if (!rc && fw) {   // weight gradients (mlp.0's first K0 columns of its ldw-wide rows)
    rc = ncf_defer(lst, workspace + T::kW0, nb, PW, N0 * K0, a.l[0].dw, 0, K0, a.l[0].ldw);
    if (!rc) rc = ncf_defer(lst, workspace + T::kW1, nb, PW, N1 * N0, a.l[1].dw, 0, N0, a.l[1].ldw);
    if (!rc) rc = ncf_defer(lst, workspace + T::kW2, nb, PW, N2 * N1, a.l[2].dw, 0, N1, a.l[2].ldw);
  }
  if (!rc && head) {
    // head partials: one reduction when the flat gradient buffer lays the six head parameters
    // out like the partial row, else one per parameter; the BCE sum scaled by 1/n into loss
    const float* hp = workspace + 3 * (N0 + N1 + N2);   // (within each partial row)
    float* base = h.grad_mf_out_w;
    const bool flat = h.grad_mf_out_b == base + T::kHmfB && h.grad_mlp_out_w == base + T::kHmlW &&
                      h.grad_mlp_out_b == base + T::kHmlB && h.grad_final_w == base + T::kHfW &&
                      h.grad_final_b == base + T::kHfB;
    if (flat) {
      rc = ncf_defer(lst, hp, nb, PW, T::kHfB + 1, base, 0, T::kHfB + 1, T::kHfB + 1);
    } else {
      rc = ncf_defer(lst, hp + T::kHmfW, nb, PW, K0, h.grad_mf_out_w, 0, K0, K0);
      if (!rc) rc = ncf_defer(lst, hp + T::kHmfB, nb, PW, 1, h.grad_mf_out_b, 0, 1, 1);
      if (!rc) rc = ncf_defer(lst, hp + T::kHmlW, nb, PW, N2, h.grad_mlp_out_w, 0, N2, N2);
      if (!rc) rc = ncf_defer(lst, hp + T::kHmlB, nb, PW, 1, h.grad_mlp_out_b, 0, 1, 1);
      if (!rc) rc = ncf_defer(lst, hp + T::kHfW, nb, PW, 2, h.grad_final_w, 0, 2, 2);
      if (!rc) rc = ncf_defer(lst, hp + T::kHfB, nb, PW, 1, h.grad_final_b, 0, 1, 1);
    }
    if (!rc && h.loss) rc = ncf_defer(lst, hp + T::kHloss, nb, PW, 1, h.loss, 0, 1, 1, inv_n);
  }
  return rc;
}

}  // namespace
}  // namespace ncf_mlp
