// Batched deterministic reductions: every deferred gradient reduction of a backward pass in two
// launches (ncf_hip.h, "deferred reductions").
//
// A training step produces ~25 parameter gradients as sums over batch rows (split-K slabs of the
// weight gradients, per-block dgamma/dbeta/dbias partials of the row ops, the head and the
// embedding LayerNorms).  None of them is on the critical path of the backward (only dX is), so
// instead of two small launches each, the list is run at the end of the backward:
//   stage 1: one 256-thread block per (descriptor, 64 outputs, chunk of <= 64 partials); a
//            descriptor with P <= NCF_REDUCE_ONE_STAGE (256) partials finishes here, otherwise
//            each chunk writes its own row of `scratch`;
//   stage 2: sums the chunk rows of the multi-chunk descriptors in chunk order.
// The summation order of every output depends only on (P, chunking) — never on scheduling —
// and is the order of ncf_reduce_parts (ncf_common.h), so a deferred reduction is bit-identical
// to the inline one.
#include "ncf_common.h"

namespace {

constexpr int kPB = 64;          // partials per stage-1 chunk
constexpr int kMaxPerLaunch = 24; // descriptors per launch (kernel-argument size)
// ncf_reduce_set_vec: 0 one column per lane, 1 four columns per lane (16-byte loads, 16 in
// flight per thread; the default), 2 the same with 32 in flight per thread (two chunk
// iterations' loads issued together).  2 measured neutral (run r06zk, 3 interleaved runs each:
// C2 min 0.2652 against 0.2660 ms/step, the batch's reductions 36.1 against 36.9 us; B = 256
// 14.8 against 12.6 us): the ~5 waves per CU of the grid already keep enough bytes in flight
int VEC_LANES = 1;

struct BatchArgs {
  ncf_reduce_desc d[kMaxPerLaunch];
  int64_t scr[kMaxPerLaunch];        // scratch offset (floats) of multi-chunk descriptors
  uint32_t first[kMaxPerLaunch + 1]; // first block of descriptor i (prefix over blocks)
  int32_t chunks[kMaxPerLaunch];
  int32_t vec[kMaxPerLaunch];        // 16-byte (four-column) lanes
  int32_t count;
};

__device__ __forceinline__ int find_desc(const BatchArgs& a, uint32_t b) {
  int i = 0;
  while (i + 1 < a.count && a.first[i + 1] <= b) ++i;
  return i;
}

__device__ __forceinline__ void store_out(const ncf_reduce_desc& d, int64_t i, float t) {
  float* o = d.out + (i / d.cols) * d.ldo + (i % d.cols);
  const float v = d.scale * t;
  *o = d.accumulate ? *o + v : v;
}

template <typename T> __device__ __forceinline__ T zero();
template <> __device__ __forceinline__ float zero<float>() { return 0.0f; }
template <> __device__ __forceinline__ float4 zero<float4>() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// Stage-1 sum of wave w's partials (rows pb + w, pb + w + 4, ... < pe) at element(s) i: T = float
// (one column per lane) or float4 (four adjacent columns per lane, 16-byte loads: each column's
// additions are the scalar form's, in the same order — the same bits).
template <typename T, bool DEEP = false>
__device__ __forceinline__ T stage1_sum(const float* __restrict__ part, int64_t stride, int64_t i,
                                        int pb, int pe, int w) {
  T a0 = zero<T>(), a1 = zero<T>(), a2 = zero<T>(), a3 = zero<T>();
  int p = pb + w;
  if (DEEP) {
    // 32 loads in flight (two iterations of the loop below at once; the same additions in the
    // same order: accumulator j % 4 takes partial p + 4j, j ascending)
    for (; p + 124 < pe; p += 128) {
      T v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = *(const T*)(part + (int64_t)(p + 4 * j) * stride + i);
#pragma unroll
      for (int j = 0; j < 32; j += 4) {
        a0 += v[j];
        a1 += v[j + 1];
        a2 += v[j + 2];
        a3 += v[j + 3];
      }
    }
  }
  // 16 loads in flight per thread (a full 64-partial chunk in one batch), summed in the order
  // of the loop below (accumulator j % 4 takes partial p + 4j): the same bits, without the
  // four dependent rounds of HBM latency
  for (; p + 60 < pe; p += 64) {
    T v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = *(const T*)(part + (int64_t)(p + 4 * j) * stride + i);
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      a0 += v[j];
      a1 += v[j + 1];
      a2 += v[j + 2];
      a3 += v[j + 3];
    }
  }
  for (; p + 12 < pe; p += 16) {
    a0 += *(const T*)(part + (int64_t)p * stride + i);
    a1 += *(const T*)(part + (int64_t)(p + 4) * stride + i);
    a2 += *(const T*)(part + (int64_t)(p + 8) * stride + i);
    a3 += *(const T*)(part + (int64_t)(p + 12) * stride + i);
  }
  for (; p < pe; p += 4) a0 += *(const T*)(part + (int64_t)p * stride + i);
  return (a0 + a1) + (a2 + a3);
}

// One 256-thread block per (descriptor, 64 lanes of columns, chunk of <= 64 partials); a
// descriptor flagged vec (a.vec: L, stride and the partial base 16-byte multiples) takes four
// columns per lane — 256 per block, 16-byte loads (stage 1 streams the batch's ~76 MB of
// weight-gradient partial sets at C2: the wide loads carry it nearer the HBM rate).
__global__ __launch_bounds__(256) void k_reduce_batch1(const BatchArgs a, float* __restrict__ scratch) {
  __shared__ float4 red[4][64];
  const int di = find_desc(a, blockIdx.x);
  const ncf_reduce_desc& d = a.d[di];
  const int ch = a.chunks[di];
  const bool vec = a.vec[di] != 0;
  const bool deep = a.vec[di] == 2;
  const int vw = vec ? 4 : 1;
  const uint32_t local = blockIdx.x - a.first[di];
  const uint32_t gx = (uint32_t)((d.L + 64 * vw - 1) / (64 * vw));
  const int64_t i = ((int64_t)(local % gx) * 64 + (threadIdx.x & 63)) * vw;
  const int y = (int)(local / gx);
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  const int pb = ch > 1 ? y * kPB : 0;
  const int pe = ch > 1 ? min(d.P, pb + kPB) : d.P;
  if (vec) {
    float4 s = zero<float4>();
    if (i < d.L)
      s = deep ? stage1_sum<float4, true>(d.part, d.stride, i, pb, pe, w)
               : stage1_sum<float4>(d.part, d.stride, i, pb, pe, w);
    red[w][l] = s;
    __syncthreads();
    if (w == 0 && i < d.L) {
      const float4 t = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
      if (ch > 1) {
        *(float4*)(scratch + a.scr[di] + (int64_t)y * d.L + i) = t;
      } else {
        store_out(d, i, t.x);
        store_out(d, i + 1, t.y);
        store_out(d, i + 2, t.z);
        store_out(d, i + 3, t.w);
      }
    }
    return;
  }
  float s = 0.0f;
  if (i < d.L) s = stage1_sum<float>(d.part, d.stride, i, pb, pe, w);
  red[w][l].x = s;
  __syncthreads();
  if (w == 0 && i < d.L) {
    const float t = (red[0][l].x + red[1][l].x) + (red[2][l].x + red[3][l].x);
    if (ch > 1) scratch[a.scr[di] + (int64_t)y * d.L + i] = t;
    else store_out(d, i, t);
  }
}

// stage 2: one thread per output element (four per thread for a vec descriptor) of the
// multi-chunk descriptors
template <typename T>
__device__ __forceinline__ T stage2_sum(const float* __restrict__ s, int64_t L, int pe) {
  // k_reduce_parts' order: "wave" w sums rows w, w+4, ... with 4 accumulators, fixed combine
  T ws[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    T a0 = zero<T>(), a1 = zero<T>(), a2 = zero<T>(), a3 = zero<T>();
    int p = w;
    for (; p + 12 < pe; p += 16) {
      a0 += *(const T*)(s + (int64_t)p * L);
      a1 += *(const T*)(s + (int64_t)(p + 4) * L);
      a2 += *(const T*)(s + (int64_t)(p + 8) * L);
      a3 += *(const T*)(s + (int64_t)(p + 12) * L);
    }
    for (; p < pe; p += 4) a0 += *(const T*)(s + (int64_t)p * L);
    ws[w] = (a0 + a1) + (a2 + a3);
  }
  return (ws[0] + ws[1]) + (ws[2] + ws[3]);
}

__global__ __launch_bounds__(256) void k_reduce_batch2(const BatchArgs a,
                                                       const float* __restrict__ scratch) {
  const int di = find_desc(a, blockIdx.x);
  const ncf_reduce_desc& d = a.d[di];
  const bool vec = a.vec[di] != 0;
  const int64_t i = ((int64_t)(blockIdx.x - a.first[di]) * 256 + threadIdx.x) * (vec ? 4 : 1);
  if (i >= d.L) return;
  const float* s = scratch + a.scr[di] + i;
  const int pe = a.chunks[di];
  if (vec) {
    const float4 t = stage2_sum<float4>(s, d.L, pe);
    store_out(d, i, t.x);
    store_out(d, i + 1, t.y);
    store_out(d, i + 2, t.z);
    store_out(d, i + 3, t.w);
    return;
  }
  store_out(d, i, stage2_sum<float>(s, d.L, pe));
}

int chunks_of(int P) { return P > NCF_REDUCE_ONE_STAGE ? (P + kPB - 1) / kPB : 1; }

}  // namespace

extern "C" int64_t ncf_reduce_set_vec(int64_t on) {
  const int was = VEC_LANES;
  if (on >= 0) VEC_LANES = on > 2 ? 2 : (int)on;
  return was;
}

extern "C" int64_t ncf_reduce_batch_scratch(const ncf_reduce_list* list) {
  if (!list) return 0;
  int64_t f = 0;
  for (int i = 0; i < list->count && i < NCF_REDUCE_LIST_MAX; ++i) {
    const int c = chunks_of(list->d[i].P);
    if (c > 1) f += (int64_t)c * list->d[i].L;
  }
  return f;
}

extern "C" int ncf_reduce_batch(const ncf_reduce_list* list, float* scratch,
                                int64_t scratch_floats, void* stream) {
  NCF_CHECK_ARG(list && list->count >= 0 && list->count <= NCF_REDUCE_LIST_MAX,
                "ncf_reduce_batch: bad list");
  if (scratch_floats < ncf_reduce_batch_scratch(list)) {
    ncf_set_error("ncf_reduce_batch: scratch %lld < %lld floats", (long long)scratch_floats,
                  (long long)ncf_reduce_batch_scratch(list));
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  int64_t scr_off = 0;
  for (int base = 0; base < list->count; base += kMaxPerLaunch) {
    BatchArgs a1, a2;
    memset(&a1, 0, sizeof(a1));
    memset(&a2, 0, sizeof(a2));
    uint32_t b1 = 0, b2 = 0;
    for (int j = 0; j < kMaxPerLaunch && base + j < list->count; ++j) {
      const ncf_reduce_desc& d = list->d[base + j];
      NCF_CHECK_ARG(d.part && d.out && d.L >= 0 && d.P >= 1 && d.cols >= 1 && d.stride >= d.L,
                    "ncf_reduce_batch: bad descriptor %d", base + j);
      const int c = chunks_of(d.P);
      const bool vec = VEC_LANES > 0 && d.L % 4 == 0 && d.stride % 4 == 0 &&
                       ((uintptr_t)d.part & 15) == 0 &&
                       (c == 1 || (scr_off % 4 == 0 && ((uintptr_t)scratch & 15) == 0));
      const int vw = vec ? 4 : 1;
      const uint32_t gx = (uint32_t)((d.L + 64 * vw - 1) / (64 * vw));
      a1.d[a1.count] = d;
      a1.vec[a1.count] = vec ? VEC_LANES : 0;
      a1.chunks[a1.count] = c;
      a1.first[a1.count] = b1;
      a1.scr[a1.count] = c > 1 ? scr_off : 0;
      b1 += gx * (uint32_t)c;
      if (c > 1) {
        a2.d[a2.count] = d;
        a2.chunks[a2.count] = c;
        a2.vec[a2.count] = vec;
        a2.first[a2.count] = b2;
        a2.scr[a2.count] = scr_off;
        b2 += (uint32_t)((d.L + 256 * vw - 1) / (256 * vw));
        ++a2.count;
        scr_off += (int64_t)c * d.L;
      }
      ++a1.count;
    }
    a1.first[a1.count] = b1;
    a2.first[a2.count] = b2;
    if (b1 > 0) {
      hipLaunchKernelGGL(k_reduce_batch1, dim3(b1), dim3(256), 0, st, a1, scratch);
      NCF_CHECK_LAUNCH("ncf_reduce_batch(stage 1)");
    }
    if (b2 > 0) {
      hipLaunchKernelGGL(k_reduce_batch2, dim3(b2), dim3(256), 0, st, a2, (const float*)scratch);
      NCF_CHECK_LAUNCH("ncf_reduce_batch(stage 2)");
    }
  }
  return NCF_OK;
}
