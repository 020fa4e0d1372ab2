// Shared device/host helpers for the MI355X (gfx950, CDNA4) AdvancedNCF kernels.
// Everything here is wave64-native: cross-lane reductions use 64-lane shuffles, and a
// "row group" of L lanes (L = D/4, float4 per lane) reduces with xor-shuffles inside the group.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#include "ncf_hip.h"  // the public C-ABI: every extern "C" definition is checked against it

#define NCF_WAVE 64

// ---------------------------------------------------------------- error handling (host)
// Thread-local last-error string exposed through ncf_last_error().
void ncf_set_error(const char* fmt, ...);

// NCF_OK / NCF_ERR_ARG (bad shape, pointer, unsupported size) / NCF_ERR_LAUNCH (hip launch
// failure) / NCF_ERR_WORKSPACE (workspace too small) come from ncf_hip.h

#define NCF_CHECK_ARG(cond, ...)                 \
  do {                                           \
    if (!(cond)) {                               \
      ncf_set_error(__VA_ARGS__);                \
      return NCF_ERR_ARG;                        \
    }                                            \
  } while (0)

// NCF_DEBUG_SYNC=1 (fault triage only): every launch is followed by a device synchronise, so
// a kernel that faults is named by the launch that raised it (printed to stderr).
static inline bool ncf_debug_sync() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("NCF_DEBUG_SYNC");
    on = (e && e[0] == '1') ? 1 : 0;
  }
  return on != 0;
}

#define NCF_CHECK_LAUNCH(name)                                                   \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ == hipSuccess && ncf_debug_sync()) {                                  \
      e_ = hipDeviceSynchronize();                                               \
      if (e_ != hipSuccess) {                                                    \
        fprintf(stderr, "NCF_DEBUG_SYNC: %s: %s\n", name, hipGetErrorString(e_)); \
        fflush(stderr);                                                          \
      }                                                                          \
    }                                                                            \
    if (e_ != hipSuccess) {                                                      \
      ncf_set_error("%s: launch failed: %s", name, hipGetErrorString(e_));       \
      return NCF_ERR_LAUNCH;                                                     \
    }                                                                            \
  } while (0)

static inline int ncf_cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------- device helpers
template <int L>
__device__ __forceinline__ float group_sum(float v) {
  // sum over an aligned group of L lanes (L power of two <= 64)
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) { return group_sum<64>(v); }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// ---- bf16 embedding tables (the C2 "bf16" configuration: tables bf16, Adam moments fp32).
// A bf16 value is the high half of the fp32 with the same leading bits; fp32 -> bf16 rounds to
// nearest even (NaN kept quiet).  Table kernels templated on BF read / write their parameter
// rows through ldp/stp (element index i of a float* that really points at bf16 when BF).
__device__ __forceinline__ float ncf_bf2f(uint32_t h) { return __uint_as_float(h << 16); }
// one v_cvt_pk_bf16_f32 (IEEE round to nearest even) on gfx950
__device__ __forceinline__ uint32_t ncf_f2bf(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
__device__ __forceinline__ float ncf_round_bf16(float f) { return (float)(__bf16)f; }
template <bool BF>
__device__ __forceinline__ float ldp(const float* p, int64_t i) {
  if constexpr (BF) return ncf_bf2f(reinterpret_cast<const uint16_t*>(p)[i]);
  else return p[i];
}
template <bool BF>
__device__ __forceinline__ void stp(float* p, int64_t i, float v) {
  if constexpr (BF) reinterpret_cast<uint16_t*>(p)[i] = (uint16_t)ncf_f2bf(v);
  else p[i] = v;
}
template <bool BF>
__device__ __forceinline__ float4 ldp4(const float* p, int64_t i) {   // i: multiple of 4
  if constexpr (BF) {
    const uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p) + i);
    return make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                       __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u));
  } else {
    return ld4(p + i);
  }
}
template <bool BF>
__device__ __forceinline__ void stp4(float* p, int64_t i, float4 v) {
  if constexpr (BF) {
    uint2 r;
    r.x = ncf_f2bf(v.x) | (ncf_f2bf(v.y) << 16);
    r.y = ncf_f2bf(v.z) | (ncf_f2bf(v.w) << 16);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p) + i) = r;
  } else {
    st4(p + i, v);
  }
}

// Counter-based dropout RNG: a 64-bit mix of (seed, element index) -> uniform [0,1).
// Deterministic per (seed, index); independent of launch geometry.
// Dropout keep decisions.  One 64-bit hash (ncf_drop_bits) of (seed, idx / 4) yields four 16-bit uniforms,
// field idx % 4 decides element idx: keep iff u >= round(p * 65536) (keep probability 1 - p to
// 1/65536).  A float4-aligned group of four elements costs a single hash.
__device__ __forceinline__ uint64_t ncf_hash64(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t ncf_drop_threshold(float p) {
  return (uint32_t)(p * 65536.0f + 0.5f);
}

// 32-bit avalanche mixer (two multiply-xorshift rounds; full avalanche, low bias)
__device__ __forceinline__ uint32_t ncf_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// the 64 dropout bits of float4 group idx4: two 32-bit mixes of the group index under keys
// derived from the 64-bit seed (and the index's high word).  32-bit multiplies only: the
// 64-bit splitmix of ncf_hash64 costs ~2.5x the VALU work, and the dropout masks are
// recomputed in every LayerNorm of the tower, forward and backward.
__device__ __forceinline__ uint64_t ncf_drop_bits(uint64_t seed, uint64_t idx4) {
  const uint32_t k = (uint32_t)seed ^ ncf_mix32((uint32_t)(seed >> 32) ^ (uint32_t)(idx4 >> 32));
  const uint32_t i = (uint32_t)idx4;
  const uint32_t h0 = ncf_mix32(i ^ k), h1 = ncf_mix32(i ^ k ^ 0x9E3779B9u);
  return ((uint64_t)h1 << 32) | h0;
}

// keep-scale of element idx for dropout probability p (nn.Dropout: scale 1/(1-p))
__device__ __forceinline__ float ncf_dropout_scale(uint64_t seed, uint64_t idx, float p, float inv_keep) {
  const uint32_t u = (uint32_t)(ncf_drop_bits(seed, idx >> 2) >> (16 * (idx & 3))) & 0xFFFFu;
  return u >= ncf_drop_threshold(p) ? inv_keep : 0.0f;
}

// keep-scales of elements idx4*4 .. idx4*4+3 (same decisions as ncf_dropout_scale)
__device__ __forceinline__ float4 ncf_dropout_scale4(uint64_t seed, uint64_t idx4, float p, float inv_keep) {
  const uint64_t z = ncf_drop_bits(seed, idx4);
  const uint32_t t = ncf_drop_threshold(p);
  return make_float4((uint32_t)(z & 0xFFFFu) >= t ? inv_keep : 0.0f,
                     (uint32_t)((z >> 16) & 0xFFFFu) >= t ? inv_keep : 0.0f,
                     (uint32_t)((z >> 32) & 0xFFFFu) >= t ? inv_keep : 0.0f,
                     (uint32_t)(z >> 48) >= t ? inv_keep : 0.0f);
}

// out[i] (+)= sum_z part[z*stride + i] over z = 0..parts-1 in order (deterministic, no atomics)
template <int Dummy = 0>
__global__ void k_sum_partials(const float* __restrict__ part, int parts, int64_t stride, int64_t n,
                               float* __restrict__ out, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.0f;
  for (int z = 0; z < parts; ++z) s += part[(int64_t)z * stride + i];
  out[i] = accumulate ? out[i] + s : s;
}

// Deterministic parallel reduction of P partial rows:
//   out[(i / cols) * ldo + i % cols] (+)= sum_{p < P} part[p * stride + i],  i < L
// One 256-thread block per 64 consecutive i and per chunk of PB partials (blockIdx.y); wave w
// sums p = w, w+4, ... (4-way unrolled, several loads in flight per lane); the 4 wave sums are
// combined in fixed order in LDS.  With gridDim.y > 1 each chunk writes its own output row
// (out + y * L, dense) and a second launch sums the chunks — always the same order.
template <int Dummy = 0>
__global__ __launch_bounds__(256) void k_reduce_parts(const float* __restrict__ part, int P,
                                                      int PB, int64_t stride, int64_t L,
                                                      float* __restrict__ out, int accumulate,
                                                      int64_t cols, int64_t ldo) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  const int pb = blockIdx.y * PB;
  const int pe = min(P, pb + PB);
  float s = 0.0f;
  if (i < L) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int p = pb + w;
    for (; p + 12 < pe; p += 16) {
      a0 += part[(int64_t)p * stride + i];
      a1 += part[(int64_t)(p + 4) * stride + i];
      a2 += part[(int64_t)(p + 8) * stride + i];
      a3 += part[(int64_t)(p + 12) * stride + i];
    }
    for (; p < pe; p += 4) a0 += part[(int64_t)p * stride + i];
    s = (a0 + a1) + (a2 + a3);
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && i < L) {
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    if (gridDim.y > 1) {
      out[(int64_t)blockIdx.y * L + i] = t;
    } else {
      float* o = out + (i / cols) * ldo + (i % cols);
      *o = accumulate ? *o + t : t;
    }
  }
}

constexpr int NCF_REDUCE_PB = 64;
// up to this many partials reduce in ONE stage (4 waves x 64 partials per output column); more
// take two stages (chunks of NCF_REDUCE_PB, then the chunk rows).  256 covers the C2 step's
// per-workgroup partial sets (256 tower / attention workgroups), so its reductions need no
// second launch (was 2 x NCF_REDUCE_PB = 128)
constexpr int NCF_REDUCE_ONE_STAGE = 256;

// scratch floats needed by ncf_reduce_parts for P partials of length L
static inline int64_t ncf_reduce_scratch(int P, int64_t L) {
  return P > NCF_REDUCE_ONE_STAGE ? (int64_t)((P + NCF_REDUCE_PB - 1) / NCF_REDUCE_PB) * L : 0;
}

// Reduce P partial rows; two deterministic stages when P is large (needs `scratch` of
// ncf_reduce_scratch(P, L) floats; with scratch == nullptr a single stage is used).
static inline void ncf_reduce_parts(const float* part, int P, int64_t stride, int64_t L, float* out,
                                    int accumulate, int64_t cols, int64_t ldo, hipStream_t st,
                                    float* scratch = nullptr) {
  if (L <= 0) return;
  const unsigned gx = (unsigned)((L + 63) / 64);
  if (scratch && P > NCF_REDUCE_ONE_STAGE) {
    const int chunks = (P + NCF_REDUCE_PB - 1) / NCF_REDUCE_PB;
    hipLaunchKernelGGL(k_reduce_parts<>, dim3(gx, chunks), dim3(256), 0, st, part, P,
                       NCF_REDUCE_PB, stride, L, scratch, 0, L, L);
    hipLaunchKernelGGL(k_reduce_parts<>, dim3(gx, 1), dim3(256), 0, st, scratch, chunks, chunks,
                       L, L, out, accumulate, cols, ldo);
    return;
  }
  hipLaunchKernelGGL(k_reduce_parts<>, dim3(gx, 1), dim3(256), 0, st, part, P, P, stride, L, out,
                     accumulate, cols, ldo);
}

// Append one reduction to a caller's deferred list (ncf_hip.h, "deferred reductions").
static inline int ncf_defer(ncf_reduce_list* l, const float* part, int64_t P, int64_t stride,
                            int64_t L, float* out, int accumulate, int64_t cols, int64_t ldo,
                            float scale = 1.0f) {
  if (L <= 0) return NCF_OK;
  if (l->count < 0 || l->count >= NCF_REDUCE_LIST_MAX) {
    ncf_set_error("deferred reduction list full (%d entries)", NCF_REDUCE_LIST_MAX);
    return NCF_ERR_ARG;
  }
  ncf_reduce_desc& d = l->d[l->count++];
  d.part = part;
  d.out = out;
  d.stride = stride;
  d.ldo = ldo;
  d.L = (int32_t)L;
  d.cols = (int32_t)cols;
  d.P = (int32_t)P;
  d.accumulate = accumulate;
  d.scale = scale;
  d.reserved = 0;
  return NCF_OK;
}
