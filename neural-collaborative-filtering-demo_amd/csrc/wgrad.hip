// Grouped weight gradients: every dW = dYᵀ·X (+ bias gradient = column sums of dY) of a training
// step in ONE launch.
//
// Reference: the backward of each nn.Linear of the attention projections (src/model/
// architecture.py:40-42, :57) and of the MLP tower (:230-246) produces grad_weight =
// grad_outputᵀ · input summed over the batch rows (and grad_bias = its row sums).  These products
// are off the backward's critical path (only dX is on it), so the engine collects them and issues
// this kernel once, after the last dX: one launch with ~1000 waves instead of seven split-K GEMMs
// of 60-250 waves each.
//
// Work item = (gemm g, 64x64 output tile, row slab).  A wave streams its slab's rows straight from
// global memory, both operands coalesced: MFMA step s covers rows r = 2s + h (h = lane half), lane
// i reads dY[r][tile_i + i] and X[r][tile_j + i] — 32 consecutive floats per half-wave — for the
// two A and two B fragments of its 2x2 v_mfma_f32_32x32x2_f32 accumulators.  Rows past the slab
// and columns past the matrix read a clamped address and are zeroed by select (no branches, so
// the unrolled loads stay in flight).  Each wave writes its 64x64 slab partial (and, for tile
// column 0, the slab's bias partial); the fixed-order slab sums are deferred reductions
// (ncf_reduce_batch): bitwise reproducible.
#include "ncf_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMaxG = NCF_WGRAD_GROUP_MAX;
constexpr int kUnroll = 8;  // MFMA steps (16 rows) per pipeline stage

struct GroupArgs {
  ncf_wgrad_desc d[kMaxG];
  float* part[kMaxG];       // slab s at part + s*stride: [m_out][k_in] weight, then [m_out] bias
  int64_t stride[kMaxG];
  uint32_t first[kMaxG + 1];
  int32_t tiles_j[kMaxG];   // 64-wide tiles along k_in
  int32_t tiles[kMaxG];     // tiles per slab
  int32_t rows_per_slab[kMaxG];
  int32_t count;
};

__device__ __forceinline__ int find_g(const GroupArgs& a, uint32_t w) {
  int g = 0;
  while (g + 1 < a.count && a.first[g + 1] <= w) ++g;
  return g;
}

__global__ __launch_bounds__(256) void k_wgrad_grouped(const GroupArgs a) {
  const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= a.first[a.count]) return;
  const int g = find_g(a, wid);
  const ncf_wgrad_desc& d = a.d[g];
  const uint32_t local = wid - a.first[g];
  const int slab = (int)(local / a.tiles[g]);
  const int t = (int)(local % a.tiles[g]);
  const int ti = t / a.tiles_j[g], tj = t % a.tiles_j[g];
  const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
  const int r0 = slab * a.rows_per_slab[g];
  const int r1 = min(d.n, r0 + a.rows_per_slab[g]);
  // per-lane columns of the two A (dY) and two B (X) fragments, clamped + validity
  const int ia0 = ti * 64 + i, ia1 = ia0 + 32, jb0 = tj * 64 + i, jb1 = jb0 + 32;
  const bool va0 = ia0 < d.m_out, va1 = ia1 < d.m_out, vb0 = jb0 < d.k_in, vb1 = jb1 < d.k_in;
  const float* pa0 = d.dy + (va0 ? ia0 : 0);
  const float* pa1 = d.dy + (va1 ? ia1 : 0);
  const float* pb0 = d.x + (vb0 ? jb0 : 0);
  const float* pb1 = d.x + (vb1 ? jb1 : 0);
  f32x16 c00, c01, c10, c11;
#pragma unroll
  for (int q = 0; q < 16; ++q) { c00[q] = 0.f; c01[q] = 0.f; c10[q] = 0.f; c11[q] = 0.f; }
  float rs0 = 0.f, rs1 = 0.f;  // bias partials (row sums of dYᵀ = column sums of dY)
  const bool want_bias = d.dbias != nullptr && tj == 0;
  // software pipeline: the loads of the next 2*kUnroll rows are issued before the MFMAs of the
  // current ones (register double buffer; sched_barrier keeps the scheduler from sinking them)
  float a0[kUnroll], a1[kUnroll], b0[kUnroll], b1[kUnroll];
  auto load = [&](int rb, float* x0, float* x1, float* y0, float* y1) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int r = rb + 2 * u + h;
      const bool vr = r < r1;
      const int64_t rr = vr ? r : r0;
      x0[u] = pa0[rr * d.ldy];
      x1[u] = pa1[rr * d.ldy];
      y0[u] = pb0[rr * d.ldx];
      y1[u] = pb1[rr * d.ldx];
      x0[u] = (vr && va0) ? x0[u] : 0.f;
      x1[u] = (vr && va1) ? x1[u] : 0.f;
      y0[u] = (vr && vb0) ? y0[u] : 0.f;
      y1[u] = (vr && vb1) ? y1[u] : 0.f;
    }
  };
  load(r0, a0, a1, b0, b1);
  for (int rb = r0; rb < r1; rb += 2 * kUnroll) {
    float n0[kUnroll], n1[kUnroll], m0[kUnroll], m1[kUnroll];
    load(rb + 2 * kUnroll < r1 ? rb + 2 * kUnroll : r0, n0, n1, m0, m1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      c00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u], b0[u], c00, 0, 0, 0);
      c01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u], b1[u], c01, 0, 0, 0);
      c10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u], b0[u], c10, 0, 0, 0);
      c11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u], b1[u], c11, 0, 0, 0);
      if (want_bias) { rs0 += a0[u]; rs1 += a1[u]; }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) { a0[u] = n0[u]; a1[u] = n1[u]; b0[u] = m0[u]; b1[u] = m1[u]; }
  }
  // slab partial [m_out][k_in]: C row (m index) = (r&3) + 8(r>>2) + 4h, column (k_in index) = i
  float* P = a.part[g] + (int64_t)slab * a.stride[g];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int m = ti * 64 + (q & 3) + 8 * (q >> 2) + 4 * h;
    if (m < d.m_out) {
      if (vb0) P[(int64_t)m * d.k_in + jb0] = c00[q];
      if (vb1) P[(int64_t)m * d.k_in + jb1] = c01[q];
    }
    if (m + 32 < d.m_out) {
      if (vb0) P[(int64_t)(m + 32) * d.k_in + jb0] = c10[q];
      if (vb1) P[(int64_t)(m + 32) * d.k_in + jb1] = c11[q];
    }
  }
  if (want_bias) {
    rs0 += __shfl_xor(rs0, 32, 64);
    rs1 += __shfl_xor(rs1, 32, 64);
    float* BP = a.part[g] + (int64_t)slab * a.stride[g] + (int64_t)d.m_out * d.k_in;
    if (h == 0) {
      if (va0) BP[ia0] = rs0;
      if (va1) BP[ia1] = rs1;
    }
  }
}

int64_t slab_rows(const ncf_wgrad_desc& d) {
  const int64_t n = d.n > 0 ? d.n : 1;
  const int64_t s = d.slabs > 0 ? d.slabs : 1;
  int64_t r = (n + s - 1) / s;
  r = (r + 2 * kUnroll - 1) / (2 * kUnroll) * (2 * kUnroll);
  return r;
}
int64_t slabs_used(const ncf_wgrad_desc& d) {
  const int64_t r = slab_rows(d);
  const int64_t n = d.n > 0 ? d.n : 1;
  return (n + r - 1) / r;
}

}  // namespace

// partials of every descriptor + the scratch of an inline (defer == NULL) reduce
extern "C" int64_t ncf_wgrad_grouped_workspace(const ncf_wgrad_desc* descs, int count) {
  int64_t f = 0, scratch = 0;
  for (int g = 0; g < count; ++g) {
    const int64_t s = slabs_used(descs[g]);
    const int64_t mn = (int64_t)descs[g].m_out * descs[g].k_in;
    f += s * (mn + (descs[g].dbias ? descs[g].m_out : 0));
    f = (f + 3) / 4 * 4;
    scratch += ncf_reduce_scratch((int)s, mn + descs[g].m_out) + ncf_reduce_scratch((int)s, descs[g].m_out);
  }
  return f + scratch;
}

extern "C" int ncf_wgrad_grouped(const ncf_wgrad_desc* descs, int count, float* workspace,
                                 int64_t workspace_floats, ncf_reduce_list* defer, void* stream) {
  NCF_CHECK_ARG(descs && count >= 0 && count <= kMaxG, "ncf_wgrad_grouped: 0..%d descriptors", kMaxG);
  if (count == 0) return NCF_OK;
  NCF_CHECK_ARG(workspace, "ncf_wgrad_grouped: null workspace");
  if (workspace_floats < ncf_wgrad_grouped_workspace(descs, count)) {
    ncf_set_error("ncf_wgrad_grouped: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  GroupArgs a;
  memset(&a, 0, sizeof(a));
  int64_t off = 0;
  uint32_t waves = 0;
  for (int g = 0; g < count; ++g) {
    const ncf_wgrad_desc& d = descs[g];
    NCF_CHECK_ARG(d.dy && d.x && d.dw && d.m_out >= 1 && d.k_in >= 1 && d.n >= 0 &&
                      d.ldy >= d.m_out && d.ldx >= d.k_in && d.ldw >= d.k_in,
                  "ncf_wgrad_grouped: bad descriptor %d", g);
    const int64_t s = slabs_used(d);
    a.d[g] = d;
    a.part[g] = workspace + off;
    a.stride[g] = (int64_t)d.m_out * d.k_in + (d.dbias ? d.m_out : 0);
    off += s * a.stride[g];
    off = (off + 3) / 4 * 4;
    a.tiles_j[g] = (int32_t)((d.k_in + 63) / 64);
    a.tiles[g] = (int32_t)(((d.m_out + 63) / 64) * a.tiles_j[g]);
    a.rows_per_slab[g] = (int32_t)slab_rows(d);
    a.first[g] = waves;
    waves += (uint32_t)(s * a.tiles[g]);
  }
  a.count = count;
  a.first[count] = waves;
  hipLaunchKernelGGL(k_wgrad_grouped, dim3((waves + 3) / 4), dim3(256), 0, st, a);
  NCF_CHECK_LAUNCH("ncf_wgrad_grouped");
  ncf_reduce_list local;
  ncf_reduce_list* lst = defer;
  if (!lst) {
    local.count = 0;
    lst = &local;
  }
  for (int g = 0; g < count; ++g) {
    const ncf_wgrad_desc& d = descs[g];
    const int64_t s = slabs_used(d);
    const int64_t mn = (int64_t)d.m_out * d.k_in;
    int rc;
    if (d.dbias && d.ldw == d.k_in && d.dbias == d.dw + mn && !d.accumulate) {
      // weight and bias adjacent in the output (a Linear's flat gradient): one reduction
      rc = ncf_defer(lst, a.part[g], s, a.stride[g], mn + d.m_out, d.dw, 0, mn + d.m_out,
                     mn + d.m_out);
    } else {
      rc = ncf_defer(lst, a.part[g], s, a.stride[g], mn, d.dw, d.accumulate, d.k_in, d.ldw);
      if (!rc && d.dbias) rc = ncf_defer(lst, a.part[g] + mn, s, a.stride[g], d.m_out, d.dbias, 0, d.m_out, d.m_out);
    }
    if (rc) return rc;
  }
  if (!defer) {
    const int64_t need = ncf_reduce_batch_scratch(lst);
    if (workspace_floats < off + need) {
      ncf_set_error("ncf_wgrad_grouped: workspace too small for the inline reduce");
      return NCF_ERR_WORKSPACE;
    }
    return ncf_reduce_batch(lst, workspace + off, workspace_floats - off, stream);
  }
  return NCF_OK;
}
