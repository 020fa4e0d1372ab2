// Shared device/host helpers for the MI355X (gfx950, CDNA4) AdvancedNCF kernels.
// Everything here is wave64-native: cross-lane reductions use 64-lane shuffles, and a
// "row group" of L lanes (L = D/4, float4 per lane) reduces with xor-shuffles inside the group.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#define NCF_WAVE 64

// ---------------------------------------------------------------- error handling (host)
// Thread-local last-error string exposed through ncf_last_error().
void ncf_set_error(const char* fmt, ...);

enum {
  NCF_OK = 0,
  NCF_ERR_ARG = -1,      // bad argument (shape / pointer / unsupported size)
  NCF_ERR_LAUNCH = -2,   // hip launch failure
  NCF_ERR_WORKSPACE = -3 // workspace too small
};

#define NCF_CHECK_ARG(cond, ...)                 \
  do {                                           \
    if (!(cond)) {                               \
      ncf_set_error(__VA_ARGS__);                \
      return NCF_ERR_ARG;                        \
    }                                            \
  } while (0)

#define NCF_CHECK_LAUNCH(name)                                                   \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
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

// Counter-based dropout RNG: a 64-bit mix of (seed, element index) -> uniform [0,1).
// Deterministic per (seed, index); independent of launch geometry.
__device__ __forceinline__ float ncf_uniform(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// keep-scale of element idx for dropout probability p (nn.Dropout: scale 1/(1-p))
__device__ __forceinline__ float ncf_dropout_scale(uint64_t seed, uint64_t idx, float p, float inv_keep) {
  return ncf_uniform(seed, idx) >= p ? inv_keep : 0.0f;
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
