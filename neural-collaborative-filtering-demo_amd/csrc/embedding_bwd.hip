// Embedding backward: sparse-gradient segment-reduce for the dual (GMF + MLP) tables, fused
// with the LayerNorm backward of mf_norm / mlp_norm.
//
// Reference: the EBC lookups (src/model/architecture.py:286-287) have dense-weight backward
// (nn.EmbeddingBag sparse=False -> `_embedding_bag_dense_backward`: index sort + accumulate
// into a fresh dense [rows, D] grad every step), preceded by the LayerNorm backward of :305-306 /
// :311-312.  Here the dense [rows, D] gradient is never materialised:
//   1. stable LSD radix sort of (id, position) pairs, users and items in the same launches
//      (blockIdx.y = id kind); 8-bit digits, passes = ceil(bits(rows)/8);
//   2. segment boundaries -> compact index c per unique id, slot[id] = c (slot maps are kept at
//      -1 between steps by ncf_slot_reset);
//   3. one L-lane group (float4 per lane) per unique id sums the upstream LN-output gradients of
//      its occurrences in position order (deterministic) and applies the LayerNorm backward ONCE:
//      LN is per-row and its backward is linear in dy, and every occurrence of an id has the same
//      input row, so sum_n LNbwd(dy_n) == LNbwd(sum_n dy_n).  dgamma/dbeta partials likewise.
// Output per kind: compact grads [num_unique, D] for the GMF and MLP tables of that kind.
#include "ncf_common.h"

namespace {

constexpr int TILE = 1024;  // keys per sort block (256 threads x 4)

struct SortProblem {
  const int64_t* ids;  // input ids [n]
  int64_t rows;        // table rows (ids outside [0, rows) are clamped to 0; forward flagged them)
};

__device__ __forceinline__ uint32_t clamp_key(int64_t id, int64_t rows) {
  return (id < 0 || id >= rows) ? 0u : (uint32_t)id;
}

// ---- pass kernels ---------------------------------------------------------------------------
// hist[kind][digit][block]
__global__ __launch_bounds__(256) void k_hist(const uint32_t* __restrict__ keys0,
                                              const uint32_t* __restrict__ keys1, int64_t n0,
                                              int64_t n1, int shift, int nb,
                                              uint32_t* __restrict__ hist) {
  __shared__ uint32_t cnt[256];
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  const uint32_t* keys = kind ? keys1 : keys0;
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TILE;
  for (int r = 0; r < 4; ++r) {
    const int64_t i = base + r * 256 + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[((int64_t)kind * 256 + threadIdx.x) * nb + blockIdx.x] = cnt[threadIdx.x];
}

// exclusive scan of hist[kind][*] (256*nb entries) in place; one 1024-thread block per kind
__global__ __launch_bounds__(1024) void k_scan_u32(uint32_t* __restrict__ data, int64_t len,
                                                   uint32_t* __restrict__ totals) {
  __shared__ uint32_t sh[1024];
  __shared__ uint32_t carry;
  uint32_t* d = data + (int64_t)blockIdx.x * len;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < len; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const uint32_t v = i < len ? d[i] : 0u;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const uint32_t x = threadIdx.x >= off ? sh[threadIdx.x - off] : 0u;
      __syncthreads();
      sh[threadIdx.x] += x;
      __syncthreads();
    }
    const uint32_t incl = sh[threadIdx.x];
    if (i < len) d[i] = carry + incl - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += incl;
    __syncthreads();
  }
  if (threadIdx.x == 0 && totals) totals[blockIdx.x] = carry;
}

// stable scatter of one pass.  Wave w owns keys [base + 256w, base + 256w + 256), processed as
// 4 ordered iterations of 64 consecutive keys; ranks inside an iteration come from 8 ballots
// (lanes with equal digit), across iterations from per-wave digit counters in LDS, across waves
// from an LDS prefix, across blocks from the scanned histogram.
__global__ __launch_bounds__(256) void k_scatter(const uint32_t* __restrict__ k_in0,
                                                 const uint32_t* __restrict__ v_in0,
                                                 const uint32_t* __restrict__ k_in1,
                                                 const uint32_t* __restrict__ v_in1, int64_t n0,
                                                 int64_t n1, int shift, int nb,
                                                 const uint32_t* __restrict__ offs,
                                                 uint32_t* __restrict__ k_out0,
                                                 uint32_t* __restrict__ v_out0,
                                                 uint32_t* __restrict__ k_out1,
                                                 uint32_t* __restrict__ v_out1) {
  __shared__ uint32_t wcnt[4][256];
  const int kind = blockIdx.y;
  const uint32_t* kin = kind ? k_in1 : k_in0;
  const uint32_t* vin = kind ? v_in1 : v_in0;
  uint32_t* kout = kind ? k_out1 : k_out0;
  uint32_t* vout = kind ? v_out1 : v_out0;
  const int64_t n = kind ? n1 : n0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int d = threadIdx.x; d < 1024; d += 256) (&wcnt[0][0])[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TILE + w * 256;
  uint32_t key[4], val[4], dig[4], loc[4];
  bool ok[4];
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int64_t i = base + it * 64 + lane;
    ok[it] = i < n;
    key[it] = ok[it] ? kin[i] : 0u;
    val[it] = ok[it] ? vin[i] : 0u;
    dig[it] = (key[it] >> shift) & 255u;
    uint64_t peers = __ballot(ok[it]);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((dig[it] >> b) & 1u);
      peers &= ((dig[it] >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t before = (uint32_t)__popcll(peers & lt);
    uint32_t c = 0;
    if (ok[it]) c = wcnt[w][dig[it]];
    __builtin_amdgcn_wave_barrier();
    loc[it] = c + before;
    const bool leader = ok[it] && before == 0;
    if (leader) wcnt[w][dig[it]] = c + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // wave prefix per digit: thread t owns digit t
  {
    const int d = threadIdx.x;
    uint32_t run = 0;
    for (int ww = 0; ww < 4; ++ww) {
      const uint32_t c = wcnt[ww][d];
      wcnt[ww][d] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    if (!ok[it]) continue;
    const uint32_t pos = offs[((int64_t)kind * 256 + dig[it]) * nb + blockIdx.x] + wcnt[w][dig[it]] + loc[it];
    kout[pos] = key[it];
    vout[pos] = val[it];
  }
}

__global__ void k_init_keys(const int64_t* __restrict__ ids0, int64_t rows0,
                            const int64_t* __restrict__ ids1, int64_t rows1, int64_t n0,
                            int64_t n1, uint32_t* __restrict__ k0, uint32_t* __restrict__ v0,
                            uint32_t* __restrict__ k1, uint32_t* __restrict__ v1) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n0) {
    k0[i] = clamp_key(ids0[i], rows0);
    v0[i] = (uint32_t)i;
  }
  if (i < n1) {
    k1[i] = clamp_key(ids1[i], rows1);
    v1[i] = (uint32_t)i;
  }
}

// ---- segments -------------------------------------------------------------------------------
// per-tile count of segment heads -> cnt[kind][block]
__global__ __launch_bounds__(256) void k_seg_count(const uint32_t* __restrict__ sk0,
                                                   const uint32_t* __restrict__ sk1, int64_t n0,
                                                   int64_t n1, int nb, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s;
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  const uint32_t* sk = kind ? sk1 : sk0;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  uint32_t c = 0;
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
    if (i < n && (i == 0 || sk[i] != sk[i - 1])) ++c;
  }
  atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0) cnt[(int64_t)kind * nb + blockIdx.x] = s;
}

// assign compact indices: segment c starts at seg_start[c]; uniq[c] = id; slot[id] = c
__global__ __launch_bounds__(256) void k_seg_assign(const uint32_t* __restrict__ sk0,
                                                    const uint32_t* __restrict__ sk1, int64_t n0,
                                                    int64_t n1, int nb,
                                                    const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ totals,
                                                    uint32_t* __restrict__ start0,
                                                    uint32_t* __restrict__ start1,
                                                    int64_t* __restrict__ uniq0,
                                                    int64_t* __restrict__ uniq1,
                                                    int32_t* __restrict__ slot0,
                                                    int32_t* __restrict__ slot1) {
  __shared__ uint32_t wsum[16];
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  const uint32_t* sk = kind ? sk1 : sk0;
  uint32_t* start = kind ? start1 : start0;
  int64_t* uniq = kind ? uniq1 : uniq0;
  int32_t* slot = kind ? slot1 : slot0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // position p = block*TILE + r*256 + tid: order by (r, w, lane) matches p order
  bool head[4];
  uint32_t rank[4];
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
    head[r] = i < n && (i == 0 || sk[i] != sk[i - 1]);
    const uint64_t m = __ballot(head[r]);
    rank[r] = (uint32_t)__popcll(m & lt);
    if (lane == 0) wsum[r * 4 + w] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  uint32_t base = off[(int64_t)kind * nb + blockIdx.x];
  for (int r = 0; r < 4; ++r) {
    uint32_t pre = 0;
    for (int q = 0; q < r * 4 + w; ++q) pre += wsum[q];
    if (head[r]) {
      const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
      const uint32_t c = base + pre + rank[r];
      start[c] = (uint32_t)i;
      uniq[c] = (int64_t)sk[i];
      if (slot) slot[sk[i]] = (int32_t)c;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) start[totals[kind]] = (uint32_t)n;
}

// One WAVE per unique id (grid-stride over c).  The wave's S = 64/L sub-groups of L = D/4 lanes
// split the id's occurrences round-robin (two loads in flight per sub-group per table), then a
// fixed xor-tree over the sub-groups combines them (deterministic), so a hot id with hundreds of
// occurrences costs ~len/(2S) load round trips instead of len.  Partial dgamma/dbeta per block:
// part[kind*nbr + block][0:D mf_g | D:2D mf_b | 2D:3D mlp_g | 3D:4D mlp_b]
template <int D>
__global__ __launch_bounds__(256) void k_seg_reduce_ln(
    const uint32_t* __restrict__ sv0, const uint32_t* __restrict__ sv1,
    const uint32_t* __restrict__ start0, const uint32_t* __restrict__ start1,
    const int64_t* __restrict__ uniq0, const int64_t* __restrict__ uniq1,
    const uint32_t* __restrict__ totals, const float* __restrict__ dy_mf0,
    const float* __restrict__ dy_mlp0, const float* __restrict__ dy_mf1,
    const float* __restrict__ dy_mlp1, const float* __restrict__ t_mf0,
    const float* __restrict__ t_mlp0, const float* __restrict__ t_mf1,
    const float* __restrict__ t_mlp1, const float* __restrict__ g_mf,
    const float* __restrict__ g_mlp, float eps, float* __restrict__ G_mf0,
    float* __restrict__ G_mlp0, float* __restrict__ G_mf1, float* __restrict__ G_mlp1,
    float* __restrict__ part) {
  constexpr int L = D / 4;
  constexpr int S = 64 / L;  // sub-groups per wave
  __shared__ __attribute__((aligned(16))) float red[4][4 * D];
  const int kind = blockIdx.y;
  const uint32_t* sv = kind ? sv1 : sv0;
  const uint32_t* start = kind ? start1 : start0;
  const int64_t* uniq = kind ? uniq1 : uniq0;
  const float* dmf = kind ? dy_mf1 : dy_mf0;
  const float* dml = kind ? dy_mlp1 : dy_mlp0;
  const float* tmf = kind ? t_mf1 : t_mf0;
  const float* tml = kind ? t_mlp1 : t_mlp0;
  float* Gmf = kind ? G_mf1 : G_mf0;
  float* Gml = kind ? G_mlp1 : G_mlp0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sg = lane / L, sub = lane % L;
  const int col = sub * 4;
  const int64_t U = totals[kind];
  const float4 gm = ld4(g_mf + col), gl = ld4(g_mlp + col);
  float4 a_gm = make_float4(0, 0, 0, 0), a_bm = a_gm, a_gl = a_gm, a_bl = a_gm;
  for (int64_t c = (int64_t)blockIdx.x * 4 + w; c < U; c += (int64_t)gridDim.x * 4) {
    const uint32_t s0 = start[c], s1 = start[c + 1];
    float4 sm = make_float4(0, 0, 0, 0), sl = sm, tm = sm, tl = sm;
    uint32_t k = s0 + sg;
    for (; k + S < s1; k += 2 * S) {
      const int64_t r0 = sv[k], r1 = sv[k + S];
      const float4 a0 = ld4(dmf + r0 * D + col), b0 = ld4(dml + r0 * D + col);
      const float4 a1 = ld4(dmf + r1 * D + col), b1 = ld4(dml + r1 * D + col);
      sm.x += a0.x; sm.y += a0.y; sm.z += a0.z; sm.w += a0.w;
      sl.x += b0.x; sl.y += b0.y; sl.z += b0.z; sl.w += b0.w;
      tm.x += a1.x; tm.y += a1.y; tm.z += a1.z; tm.w += a1.w;
      tl.x += b1.x; tl.y += b1.y; tl.z += b1.z; tl.w += b1.w;
    }
    if (k < s1) {
      const int64_t r0 = sv[k];
      const float4 a0 = ld4(dmf + r0 * D + col), b0 = ld4(dml + r0 * D + col);
      sm.x += a0.x; sm.y += a0.y; sm.z += a0.z; sm.w += a0.w;
      sl.x += b0.x; sl.y += b0.y; sl.z += b0.z; sl.w += b0.w;
    }
    sm.x += tm.x; sm.y += tm.y; sm.z += tm.z; sm.w += tm.w;
    sl.x += tl.x; sl.y += tl.y; sl.z += tl.z; sl.w += tl.w;
#pragma unroll
    for (int o = L; o < 64; o <<= 1) {  // combine sub-groups (same columns, lanes L apart)
      sm.x += __shfl_xor(sm.x, o, 64); sm.y += __shfl_xor(sm.y, o, 64);
      sm.z += __shfl_xor(sm.z, o, 64); sm.w += __shfl_xor(sm.w, o, 64);
      sl.x += __shfl_xor(sl.x, o, 64); sl.y += __shfl_xor(sl.y, o, 64);
      sl.z += __shfl_xor(sl.z, o, 64); sl.w += __shfl_xor(sl.w, o, 64);
    }
    const int64_t id = uniq[c];
    // two LayerNorm backwards (GMF row, MLP row); every sub-group computes, sub-group 0 stores
#pragma unroll
    for (int tbl = 0; tbl < 2; ++tbl) {
      const float4 x = ld4((tbl ? tml : tmf) + id * D + col);
      const float4 dy = tbl ? sl : sm;
      const float4 gg = tbl ? gl : gm;
      const float mean = group_sum<L>(x.x + x.y + x.z + x.w) * (1.0f / D);
      const float4 xc = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
      const float var = group_sum<L>(xc.x * xc.x + xc.y * xc.y + xc.z * xc.z + xc.w * xc.w) * (1.0f / D);
      const float rstd = 1.0f / sqrtf(var + eps);
      const float4 h = make_float4(xc.x * rstd, xc.y * rstd, xc.z * rstd, xc.w * rstd);
      const float4 gd = make_float4(dy.x * gg.x, dy.y * gg.y, dy.z * gg.z, dy.w * gg.w);
      const float m1 = group_sum<L>(gd.x + gd.y + gd.z + gd.w) * (1.0f / D);
      const float m2 = group_sum<L>(gd.x * h.x + gd.y * h.y + gd.z * h.z + gd.w * h.w) * (1.0f / D);
      if (sg == 0) {
        const float4 dx = make_float4(rstd * (gd.x - m1 - h.x * m2), rstd * (gd.y - m1 - h.y * m2),
                                      rstd * (gd.z - m1 - h.z * m2), rstd * (gd.w - m1 - h.w * m2));
        st4((tbl ? Gml : Gmf) + c * D + col, dx);
        float4& ag = tbl ? a_gl : a_gm;
        float4& ab = tbl ? a_bl : a_bm;
        ag.x += dy.x * h.x; ag.y += dy.y * h.y; ag.z += dy.z * h.z; ag.w += dy.w * h.w;
        ab.x += dy.x; ab.y += dy.y; ab.z += dy.z; ab.w += dy.w;
      }
    }
  }
  if (sg == 0) {
    float* rr = red[w];
    st4(rr + col, a_gm);
    st4(rr + D + col, a_bm);
    st4(rr + 2 * D + col, a_gl);
    st4(rr + 3 * D + col, a_bl);
  }
  __syncthreads();
  float* out = part + ((int64_t)kind * gridDim.x + blockIdx.x) * 4 * D;
  for (int i = threadIdx.x; i < 4 * D; i += 256)
    out[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

__global__ void k_ln_param_scatter(const float* __restrict__ red, int D, float* gm, float* bm,
                                   float* gl, float* bl) {
  for (int i = threadIdx.x; i < 4 * D; i += blockDim.x) {
    const int q = i / D, c = i % D;
    float* dst = q == 0 ? gm : q == 1 ? bm : q == 2 ? gl : bl;
    dst[c] = red[i];
  }
}

__global__ void k_slot_reset(const int64_t* __restrict__ uniq, const uint32_t* __restrict__ totals,
                             int kind, int32_t* __restrict__ slot, int64_t max_n) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= max_n || c >= (int64_t)totals[kind]) return;
  slot[uniq[c]] = -1;
}

// ---- row sharding (multi-GPU): owner(id) = id mod W, local row = id div W ----------------------
// owner bucket keys: digit = owner for valid entries, W (sorts last) for c >= count
__global__ void k_owner_keys(const int64_t* __restrict__ uniq0, const int64_t* __restrict__ uniq1,
                             const uint32_t* __restrict__ count, int64_t n, int W,
                             uint32_t* __restrict__ k0, uint32_t* __restrict__ v0,
                             uint32_t* __restrict__ k1, uint32_t* __restrict__ v1) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  k0[i] = i < (int64_t)count[0] ? (uint32_t)(uniq0[i] % W) : (uint32_t)W;
  v0[i] = (uint32_t)i;
  k1[i] = i < (int64_t)count[1] ? (uint32_t)(uniq1[i] % W) : (uint32_t)W;
  v1[i] = (uint32_t)i;
}

// after one stable pass: send_ids[j] = uniq[perm[j]], counts[kind][d] from the scanned histogram
__global__ void k_owner_finish(const int64_t* __restrict__ uniq0, const int64_t* __restrict__ uniq1,
                               const uint32_t* __restrict__ count, const uint32_t* __restrict__ sv0,
                               const uint32_t* __restrict__ sv1, int64_t n,
                               const uint32_t* __restrict__ offs, int nb, int W,
                               int64_t* __restrict__ send0, int64_t* __restrict__ send1,
                               int32_t* __restrict__ perm0, int32_t* __restrict__ perm1,
                               int64_t* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int64_t)count[0]) { perm0[i] = (int32_t)sv0[i]; send0[i] = uniq0[sv0[i]]; }
  if (i < (int64_t)count[1]) { perm1[i] = (int32_t)sv1[i]; send1[i] = uniq1[sv1[i]]; }
  if (blockIdx.x == 0 && threadIdx.x < 2 * W) {
    const int kind = threadIdx.x / W, d = threadIdx.x % W;
    const uint32_t* o = offs + (int64_t)kind * 256 * nb;
    counts[kind * W + d] = (int64_t)(o[(int64_t)(d + 1) * nb] - o[(int64_t)d * nb]);
  }
  (void)n;
}

// inverse map of a dedup: inv[position] = compact index of its id
__global__ __launch_bounds__(256) void k_seg_inverse(const uint32_t* __restrict__ sk0,
                                                     const uint32_t* __restrict__ sk1,
                                                     const uint32_t* __restrict__ sv0,
                                                     const uint32_t* __restrict__ sv1, int64_t n0,
                                                     int64_t n1, int nb,
                                                     const uint32_t* __restrict__ off,
                                                     int64_t* __restrict__ inv0,
                                                     int64_t* __restrict__ inv1) {
  __shared__ uint32_t wsum[16];
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  const uint32_t* sk = kind ? sk1 : sk0;
  const uint32_t* sv = kind ? sv1 : sv0;
  int64_t* inv = kind ? inv1 : inv0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  bool head[4];
  uint32_t rank[4];
  const uint64_t le = (lane == 63) ? ~0ull : ((1ull << (lane + 1)) - 1);  // inclusive
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
    head[r] = i < n && (i == 0 || sk[i] != sk[i - 1]);
    const uint64_t m = __ballot(head[r]);
    rank[r] = (uint32_t)__popcll(m & le);
    if (lane == 0) wsum[r * 4 + w] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  const uint32_t base = off[(int64_t)kind * nb + blockIdx.x];
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
    if (i >= n) continue;
    uint32_t pre = 0;
    for (int q = 0; q < r * 4 + w; ++q) pre += wsum[q];
    inv[sv[i]] = (int64_t)(base + pre + rank[r]) - 1;
  }
}

// owner side: per unique local row c, sum the received gradient rows of its occurrences
// (position order = source rank, then the sender's order: deterministic); src rows are [n][2D]
// (GMF | MLP), outputs compact [U][D] per table.
template <int D>
__global__ __launch_bounds__(256) void k_seg_sum_rows(
    const uint32_t* __restrict__ sv0, const uint32_t* __restrict__ sv1,
    const uint32_t* __restrict__ start0, const uint32_t* __restrict__ start1,
    const uint32_t* __restrict__ totals, const float* __restrict__ src0,
    const float* __restrict__ src1, float* __restrict__ Ga0, float* __restrict__ Gb0,
    float* __restrict__ Ga1, float* __restrict__ Gb1) {
  constexpr int L = D / 4;
  const int kind = blockIdx.y;
  const uint32_t* sv = kind ? sv1 : sv0;
  const uint32_t* start = kind ? start1 : start0;
  const float* src = kind ? src1 : src0;
  float* Ga = kind ? Ga1 : Ga0;
  float* Gb = kind ? Gb1 : Gb0;
  const int64_t U = totals[kind];
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int sub = (int)(t % L);
  for (int64_t c = t / L; c < U; c += (int64_t)gridDim.x * blockDim.x / L) {
    float4 a = make_float4(0, 0, 0, 0), b = a;
    for (uint32_t k = start[c]; k < start[c + 1]; ++k) {
      const int64_t r = sv[k];
      const float4 x = ld4(src + r * 2 * D + sub * 4), y = ld4(src + r * 2 * D + D + sub * 4);
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
    }
    st4(Ga + c * D + sub * 4, a);
    st4(Gb + c * D + sub * 4, b);
  }
}

// rows of a shard for global ids: out[j] = (t0[id/W] | t1[id/W])
template <int D>
__global__ void k_gather_shard(const int64_t* __restrict__ ids, int64_t n, int W,
                               const float* __restrict__ t0, const float* __restrict__ t1,
                               int64_t rows, float* __restrict__ out, int* err) {
  constexpr int L = D / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t j = t / L;
  const int sub = (int)(t % L);
  if (j >= n) return;
  int64_t r = ids[j] / W;
  if (r < 0 || r >= rows) {
    if (err && sub == 0) atomicOr(err, 2);
    r = 0;
  }
  st4(out + j * 2 * D + sub * 4, ld4(t0 + r * D + sub * 4));
  st4(out + j * 2 * D + D + sub * 4, ld4(t1 + r * D + sub * 4));
}

// mini0[perm[j]] = rows[j][0:D], mini1[perm[j]] = rows[j][D:2D]   (dir = 0)
// out[j] = (mini0[perm[j]] | mini1[perm[j]])                       (dir = 1)
template <int D>
__global__ void k_perm_rows(float* __restrict__ rows, const int32_t* __restrict__ perm, int64_t n,
                            float* __restrict__ mini0, float* __restrict__ mini1, int dir) {
  constexpr int L = D / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t j = t / L;
  const int sub = (int)(t % L);
  if (j >= n) return;
  const int64_t c = perm[j];
  float* r = rows + j * 2 * D + sub * 4;
  if (dir == 0) {
    st4(mini0 + c * D + sub * 4, ld4(r));
    st4(mini1 + c * D + sub * 4, ld4(r + D));
  } else {
    st4(r, ld4(mini0 + c * D + sub * 4));
    st4(r + D, ld4(mini1 + c * D + sub * 4));
  }
}

__global__ void k_ids_div(const int64_t* __restrict__ ids, int64_t n, int W, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = ids[i] / W;
}

// ---- workspace layout -----------------------------------------------------------------------
struct WS {
  uint32_t *ka0, *va0, *ka1, *va1, *kb0, *vb0, *kb1, *vb1;
  uint32_t *hist, *segcnt, *totals, *start0, *start1;
  float* part;
  float* red_scratch;
  int nb, nbr;
};

int nb_of(int64_t n) { return n == 0 ? 1 : ncf_cdiv(n, TILE); }
int nbr_of(int64_t n, int64_t D) {
  (void)D;
  int64_t b = (n + 3) / 4;  // 4 waves (segments) per block
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

int64_t ws_bytes(int64_t n, int64_t D) {
  const int nb = nb_of(n), nbr = nbr_of(n, D);
  int64_t b = 0;
  b += 8 * (n + 64) * 4;                 // 8 key/val buffers (padded)
  b += 2 * 256 * (int64_t)nb * 4 + 256;  // hist
  b += 2 * (int64_t)nb * 4 + 256;        // segcnt
  b += 64;                               // totals
  b += 2 * (n + 2) * 4 + 256;            // starts
  b += (2 * (int64_t)nbr + 1) * 4 * D * 4 + 256;
  b += ncf_reduce_scratch(2 * nbr, 4 * D) * 4 + 256;
  return b + 1024;
}

WS carve(void* base, int64_t n, int64_t D) {
  WS w;
  w.nb = nb_of(n);
  w.nbr = nbr_of(n, D);
  char* p = (char*)base;
  auto take = [&](int64_t bytes) {
    char* r = p;
    p += (bytes + 255) / 256 * 256;
    return r;
  };
  const int64_t kb = (n + 64) * 4;
  w.ka0 = (uint32_t*)take(kb); w.va0 = (uint32_t*)take(kb);
  w.ka1 = (uint32_t*)take(kb); w.va1 = (uint32_t*)take(kb);
  w.kb0 = (uint32_t*)take(kb); w.vb0 = (uint32_t*)take(kb);
  w.kb1 = (uint32_t*)take(kb); w.vb1 = (uint32_t*)take(kb);
  w.hist = (uint32_t*)take(2 * 256 * (int64_t)w.nb * 4);
  w.segcnt = (uint32_t*)take(2 * (int64_t)w.nb * 4);
  w.totals = (uint32_t*)take(64);
  w.start0 = (uint32_t*)take((n + 2) * 4);
  w.start1 = (uint32_t*)take((n + 2) * 4);
  w.part = (float*)take((2 * (int64_t)w.nbr + 1) * 4 * D * 4);
  w.red_scratch = (float*)take(ncf_reduce_scratch(2 * w.nbr, 4 * D) * 4 + 4);
  return w;
}

int bits_for(int64_t rows) {
  int b = 1;
  while (b < 32 && (1ll << b) < rows) ++b;
  return b;
}

template <int D>
int seg_reduce(const WS& w, const uint32_t* sv0, const uint32_t* sv1, const int64_t* uniq0,
               const int64_t* uniq1, const float* dmf0, const float* dml0, const float* dmf1,
               const float* dml1, const float* tmf0, const float* tml0, const float* tmf1,
               const float* tml1, const float* gmf, const float* gml, float eps, float* Gmf0,
               float* Gml0, float* Gmf1, float* Gml1, float* dgm, float* dbm, float* dgl,
               float* dbl, ncf_reduce_list* defer, hipStream_t st) {
  hipLaunchKernelGGL(k_seg_reduce_ln<D>, dim3(w.nbr, 2), dim3(256), 0, st, sv0, sv1, w.start0,
                     w.start1, uniq0, uniq1, w.totals, dmf0, dml0, dmf1, dml1, tmf0, tml0, tmf1,
                     tml1, gmf, gml, eps, Gmf0, Gml0, Gmf1, Gml1, w.part);
  NCF_CHECK_LAUNCH("ncf_embedding_bwd(seg_reduce)");
  if (defer) {
    float* const outs[4] = {dgm, dbm, dgl, dbl};
    for (int q = 0; q < 4; ++q) {
      const int rc = ncf_defer(defer, w.part + q * D, 2 * w.nbr, 4 * D, D, outs[q], 0, D, D);
      if (rc) return rc;
    }
    return NCF_OK;
  }
  float* red = w.part + (int64_t)2 * w.nbr * 4 * D;
  ncf_reduce_parts(w.part, 2 * w.nbr, 4 * D, 4 * D, red, 0, 4 * D, 4 * D, st, w.red_scratch);
  hipLaunchKernelGGL(k_ln_param_scatter, dim3(1), dim3(256), 0, st, red, D, dgm, dbm, dgl, dbl);
  NCF_CHECK_LAUNCH("ncf_embedding_bwd(finalize)");
  return NCF_OK;
}

}  // namespace

extern "C" int64_t ncf_embedding_bwd_workspace(int64_t n, int64_t dim) { return ws_bytes(n, dim); }

// sorted (keys, positions) after `passes` ping-pong passes
static void sorted_bufs(const WS& w, int passes, uint32_t** k0, uint32_t** v0, uint32_t** k1,
                        uint32_t** v1) {
  const bool odd = passes & 1;
  *k0 = odd ? w.kb0 : w.ka0;
  *v0 = odd ? w.vb0 : w.va0;
  *k1 = odd ? w.kb1 : w.ka1;
  *v1 = odd ? w.vb1 : w.va1;
}

static int passes_for(int64_t num_users, int64_t num_items) {
  return (bits_for(num_users > num_items ? num_users : num_items) + 7) / 8;
}

// Phase 1: stable radix sort of (id, position) for two id lists (kind 0 / kind 1, lengths n0 /
// n1) + segment heads: uniq ids per kind, num_unique[kind], optional slot maps.  The sorted
// positions and segment starts stay in `workspace` (sized for max(n0, n1)).
extern "C" int ncf_dedup_ids2(const int64_t* ids0, int64_t n0, int64_t rows0, const int64_t* ids1,
                              int64_t n1, int64_t rows1, int64_t dim, int64_t* uniq0,
                              int64_t* uniq1, int32_t* slot0, int32_t* slot1,
                              uint32_t* num_unique, void* workspace, int64_t workspace_bytes,
                              void* stream) {
  const int64_t n = n0 > n1 ? n0 : n1;
  NCF_CHECK_ARG(n0 >= 0 && n1 >= 0 && n < (1ll << 31), "ncf_dedup_ids: bad n");
  NCF_CHECK_ARG(rows0 < (1ll << 32) && rows1 < (1ll << 32), "ncf_dedup_ids: > 2^32 rows");
  if (workspace_bytes < ws_bytes(n, dim)) {
    ncf_set_error("ncf_dedup_ids: workspace %lld < %lld bytes", (long long)workspace_bytes,
                  (long long)ws_bytes(n, dim));
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  WS w = carve(workspace, n, dim);
  if (n > 0) {
    hipLaunchKernelGGL(k_init_keys, dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, ids0, rows0, ids1,
                       rows1, n0, n1, w.ka0, w.va0, w.ka1, w.va1);
    NCF_CHECK_LAUNCH("ncf_dedup_ids(init)");
  }
  const int passes = passes_for(rows0, rows1);
  uint32_t *ki0 = w.ka0, *vi0 = w.va0, *ki1 = w.ka1, *vi1 = w.va1;
  uint32_t *ko0 = w.kb0, *vo0 = w.vb0, *ko1 = w.kb1, *vo1 = w.vb1;
  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    if (n > 0) {
      hipLaunchKernelGGL(k_hist, dim3(w.nb, 2), dim3(256), 0, st, ki0, ki1, n0, n1, shift, w.nb,
                         w.hist);
      hipLaunchKernelGGL(k_scan_u32, dim3(2), dim3(1024), 0, st, w.hist, (int64_t)256 * w.nb,
                         (uint32_t*)nullptr);
      hipLaunchKernelGGL(k_scatter, dim3(w.nb, 2), dim3(256), 0, st, ki0, vi0, ki1, vi1, n0, n1,
                         shift, w.nb, w.hist, ko0, vo0, ko1, vo1);
      NCF_CHECK_LAUNCH("ncf_dedup_ids(sort)");
    }
    uint32_t* t;
    t = ki0; ki0 = ko0; ko0 = t;
    t = vi0; vi0 = vo0; vo0 = t;
    t = ki1; ki1 = ko1; ko1 = t;
    t = vi1; vi1 = vo1; vo1 = t;
  }
  hipLaunchKernelGGL(k_seg_count, dim3(w.nb, 2), dim3(256), 0, st, ki0, ki1, n0, n1, w.nb,
                     w.segcnt);
  hipLaunchKernelGGL(k_scan_u32, dim3(2), dim3(1024), 0, st, w.segcnt, (int64_t)w.nb, w.totals);
  hipLaunchKernelGGL(k_seg_assign, dim3(w.nb, 2), dim3(256), 0, st, ki0, ki1, n0, n1, w.nb,
                     w.segcnt, w.totals, w.start0, w.start1, uniq0, uniq1, slot0, slot1);
  NCF_CHECK_LAUNCH("ncf_dedup_ids(segments)");
  if (num_unique)
    (void)hipMemcpyAsync(num_unique, w.totals, 2 * sizeof(uint32_t), hipMemcpyDeviceToDevice, st);
  return NCF_OK;
}

extern "C" int ncf_dedup_ids(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                             int64_t dim, int64_t num_users, int64_t num_items,
                             int64_t* uniq_users, int64_t* uniq_items, int32_t* slot_users,
                             int32_t* slot_items, uint32_t* num_unique, void* workspace,
                             int64_t workspace_bytes, void* stream) {
  return ncf_dedup_ids2(user_ids, n, num_users, item_ids, n, num_items, dim, uniq_users,
                        uniq_items, slot_users, slot_items, num_unique, workspace,
                        workspace_bytes, stream);
}

// Phase 2: per unique id, sum the LN-output gradients of its occurrences (position order) and
// apply mf_norm / mlp_norm backward once; dgamma/dbeta of both norms.  Requires the workspace
// filled by ncf_dedup_ids for the same ids.
extern "C" int ncf_embedding_bwd_reduce(int64_t n, int64_t dim, int64_t num_users,
                                        int64_t num_items, const float* dy_mf_user,
                                        const float* dy_mlp_user, const float* dy_mf_item,
                                        const float* dy_mlp_item, const float* mf_user,
                                        const float* mlp_user, const float* mf_item,
                                        const float* mlp_item, const float* mf_gamma,
                                        const float* mlp_gamma, float eps, float* grad_mf_user,
                                        float* grad_mlp_user, float* grad_mf_item,
                                        float* grad_mlp_item, const int64_t* uniq_users,
                                        const int64_t* uniq_items, float* grad_mf_gamma,
                                        float* grad_mf_beta, float* grad_mlp_gamma,
                                        float* grad_mlp_beta, void* workspace,
                                        int64_t workspace_bytes, ncf_reduce_list* defer,
                                        void* stream) {
  NCF_CHECK_ARG(n >= 0 && n < (1ll << 31), "ncf_embedding_bwd_reduce: bad n");
  NCF_CHECK_ARG(dim == 16 || dim == 32 || dim == 64 || dim == 128 || dim == 256,
                "ncf_embedding_bwd_reduce: dim must be 16/32/64/128/256");
  if (workspace_bytes < ws_bytes(n, dim)) {
    ncf_set_error("ncf_embedding_bwd_reduce: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  WS w = carve(workspace, n, dim);
  uint32_t *k0, *v0, *k1, *v1;
  sorted_bufs(w, passes_for(num_users, num_items), &k0, &v0, &k1, &v1);
  switch (dim) {
#define SEG(DD)                                                                                   \
  case DD:                                                                                        \
    return seg_reduce<DD>(w, v0, v1, uniq_users, uniq_items, dy_mf_user, dy_mlp_user,             \
                          dy_mf_item, dy_mlp_item, mf_user, mlp_user, mf_item, mlp_item,          \
                          mf_gamma, mlp_gamma, eps, grad_mf_user, grad_mlp_user, grad_mf_item,    \
                          grad_mlp_item, grad_mf_gamma, grad_mf_beta, grad_mlp_gamma,             \
                          grad_mlp_beta, defer, st);
    SEG(16) SEG(32) SEG(64) SEG(128) SEG(256)
#undef SEG
  }
  return NCF_ERR_ARG;
}

// Both phases (dedup + reduce), with slot maps for the dense-exact table Adam.
extern "C" int ncf_embedding_bwd(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                                 int64_t dim, int64_t num_users, int64_t num_items,
                                 const float* dy_mf_user, const float* dy_mlp_user,
                                 const float* dy_mf_item, const float* dy_mlp_item,
                                 const float* mf_user, const float* mlp_user, const float* mf_item,
                                 const float* mlp_item, const float* mf_gamma,
                                 const float* mlp_gamma, float eps, float* grad_mf_user,
                                 float* grad_mlp_user, float* grad_mf_item, float* grad_mlp_item,
                                 int64_t* uniq_users, int64_t* uniq_items, int32_t* slot_users,
                                 int32_t* slot_items, uint32_t* num_unique, float* grad_mf_gamma,
                                 float* grad_mf_beta, float* grad_mlp_gamma, float* grad_mlp_beta,
                                 void* workspace, int64_t workspace_bytes, void* stream) {
  NCF_CHECK_ARG(dim == 16 || dim == 32 || dim == 64 || dim == 128 || dim == 256,
                "ncf_embedding_bwd: dim must be 16/32/64/128/256");
  int rc = ncf_dedup_ids(user_ids, item_ids, n, dim, num_users, num_items, uniq_users, uniq_items,
                         slot_users, slot_items, num_unique, workspace, workspace_bytes, stream);
  if (rc) return rc;
  return ncf_embedding_bwd_reduce(n, dim, num_users, num_items, dy_mf_user, dy_mlp_user,
                                  dy_mf_item, dy_mlp_item, mf_user, mlp_user, mf_item, mlp_item,
                                  mf_gamma, mlp_gamma, eps, grad_mf_user, grad_mlp_user,
                                  grad_mf_item, grad_mlp_item, uniq_users, uniq_items,
                                  grad_mf_gamma, grad_mf_beta, grad_mlp_gamma, grad_mlp_beta,
                                  workspace, workspace_bytes, nullptr, stream);
}

// slot[uniq[c]] = -1 for c < num_unique[kind] (restores the all -1 invariant after the update)
extern "C" int ncf_slot_reset(const int64_t* uniq, const uint32_t* num_unique, int kind,
                              int32_t* slot, int64_t max_n, void* stream) {
  if (max_n <= 0) return NCF_OK;
  hipLaunchKernelGGL(k_slot_reset, dim3(ncf_cdiv(max_n, 256)), dim3(256), 0, (hipStream_t)stream,
                     uniq, num_unique, kind, slot, max_n);
  NCF_CHECK_LAUNCH("ncf_slot_reset");
  return NCF_OK;
}

// ---- row-sharding C-ABI ---------------------------------------------------------------------
// Stable partition of the first count[kind] unique ids by owner = id mod world (world <= 255):
// send_ids in owner order, perm[j] = index of send_ids[j] in uniq, counts[kind*world + d].
extern "C" int ncf_owner_bucket(const int64_t* uniq0, const int64_t* uniq1, const uint32_t* count,
                                int64_t max_n, int world, int64_t* send0, int64_t* send1,
                                int32_t* perm0, int32_t* perm1, int64_t* counts,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  NCF_CHECK_ARG(world >= 1 && world <= 128 && max_n >= 0, "ncf_owner_bucket: bad world/size");
  if (workspace_bytes < ws_bytes(max_n, 16)) {
    ncf_set_error("ncf_owner_bucket: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  WS w = carve(workspace, max_n, 16);
  const int64_t n = max_n;
  if (n > 0) {
    hipLaunchKernelGGL(k_owner_keys, dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, uniq0, uniq1, count,
                       n, world, w.ka0, w.va0, w.ka1, w.va1);
    hipLaunchKernelGGL(k_hist, dim3(w.nb, 2), dim3(256), 0, st, w.ka0, w.ka1, n, n, 0, w.nb, w.hist);
    hipLaunchKernelGGL(k_scan_u32, dim3(2), dim3(1024), 0, st, w.hist, (int64_t)256 * w.nb,
                       (uint32_t*)nullptr);
    hipLaunchKernelGGL(k_scatter, dim3(w.nb, 2), dim3(256), 0, st, w.ka0, w.va0, w.ka1, w.va1, n, n,
                       0, w.nb, w.hist, w.kb0, w.vb0, w.kb1, w.vb1);
    hipLaunchKernelGGL(k_owner_finish, dim3(ncf_cdiv(n > 512 ? n : 512, 256)), dim3(256), 0, st,
                       uniq0, uniq1, count, w.vb0, w.vb1, n, w.hist, w.nb, world, send0, send1,
                       perm0, perm1, counts);
    NCF_CHECK_LAUNCH("ncf_owner_bucket");
  } else {
    (void)hipMemsetAsync(counts, 0, sizeof(int64_t) * 2 * world, st);
  }
  return NCF_OK;
}

// inv[position] = compact index, for the dedup held in `workspace` (ncf_dedup_ids2, same args)
extern "C" int ncf_dedup_inverse(int64_t n0, int64_t n1, int64_t rows0, int64_t rows1, int64_t dim,
                                 int64_t* inv0, int64_t* inv1, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  const int64_t n = n0 > n1 ? n0 : n1;
  if (workspace_bytes < ws_bytes(n, dim)) {
    ncf_set_error("ncf_dedup_inverse: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (n == 0) return NCF_OK;
  WS w = carve(workspace, n, dim);
  uint32_t *k0, *v0, *k1, *v1;
  sorted_bufs(w, passes_for(rows0, rows1), &k0, &v0, &k1, &v1);
  hipLaunchKernelGGL(k_seg_inverse, dim3(w.nb, 2), dim3(256), 0, (hipStream_t)stream, k0, k1, v0,
                     v1, n0, n1, w.nb, w.segcnt, inv0, inv1);
  NCF_CHECK_LAUNCH("ncf_dedup_inverse");
  return NCF_OK;
}

// per unique row of the dedup in `workspace`, sum the [n][2D] rows of its occurrences
extern "C" int ncf_segment_sum_rows(int64_t n0, int64_t n1, int64_t rows0, int64_t rows1,
                                    int64_t dim, const float* src0, const float* src1,
                                    float* ga0, float* gb0, float* ga1, float* gb1,
                                    void* workspace, int64_t workspace_bytes, void* stream) {
  const int64_t n = n0 > n1 ? n0 : n1;
  if (workspace_bytes < ws_bytes(n, dim)) {
    ncf_set_error("ncf_segment_sum_rows: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (n == 0) return NCF_OK;
  WS w = carve(workspace, n, dim);
  uint32_t *k0, *v0, *k1, *v1;
  sorted_bufs(w, passes_for(rows0, rows1), &k0, &v0, &k1, &v1);
  hipStream_t st = (hipStream_t)stream;
  const int blocks = ncf_cdiv(n * (dim / 4), 256) > 2048 ? 2048 : ncf_cdiv(n * (dim / 4), 256);
  switch (dim) {
#define SS(DD)                                                                                   \
  case DD:                                                                                       \
    hipLaunchKernelGGL(k_seg_sum_rows<DD>, dim3(blocks, 2), dim3(256), 0, st, v0, v1, w.start0,  \
                       w.start1, w.totals, src0, src1, ga0, gb0, ga1, gb1);                      \
    break;
    SS(16) SS(32) SS(64) SS(128) SS(256)
#undef SS
    default: ncf_set_error("ncf_segment_sum_rows: dim"); return NCF_ERR_ARG;
  }
  NCF_CHECK_LAUNCH("ncf_segment_sum_rows");
  return NCF_OK;
}

extern "C" int ncf_gather_shard_rows(const int64_t* ids, int64_t n, int world, const float* t0,
                                     const float* t1, int64_t rows, int64_t dim, float* out,
                                     int* err_flag, void* stream) {
  if (n <= 0) return NCF_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (dim) {
#define GS(DD)                                                                                   \
  case DD:                                                                                       \
    hipLaunchKernelGGL(k_gather_shard<DD>, dim3(ncf_cdiv(n * (DD / 4), 256)), dim3(256), 0, st,  \
                       ids, n, world, t0, t1, rows, out, err_flag);                              \
    break;
    GS(16) GS(32) GS(64) GS(128) GS(256)
#undef GS
    default: ncf_set_error("ncf_gather_shard_rows: dim"); return NCF_ERR_ARG;
  }
  NCF_CHECK_LAUNCH("ncf_gather_shard_rows");
  return NCF_OK;
}

// dir 0: scatter [n][2D] rows into mini tables at perm; dir 1: pack mini rows at perm into [n][2D]
extern "C" int ncf_perm_rows(float* rows, const int32_t* perm, int64_t n, int64_t dim, float* mini0,
                             float* mini1, int dir, void* stream) {
  if (n <= 0) return NCF_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (dim) {
#define PR(DD)                                                                                   \
  case DD:                                                                                       \
    hipLaunchKernelGGL(k_perm_rows<DD>, dim3(ncf_cdiv(n * (DD / 4), 256)), dim3(256), 0, st,     \
                       rows, perm, n, mini0, mini1, dir);                                        \
    break;
    PR(16) PR(32) PR(64) PR(128) PR(256)
#undef PR
    default: ncf_set_error("ncf_perm_rows: dim"); return NCF_ERR_ARG;
  }
  NCF_CHECK_LAUNCH("ncf_perm_rows");
  return NCF_OK;
}

extern "C" int ncf_ids_div(const int64_t* ids, int64_t n, int world, int64_t* out, void* stream) {
  if (n <= 0) return NCF_OK;
  hipLaunchKernelGGL(k_ids_div, dim3(ncf_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, ids, n,
                     world, out);
  NCF_CHECK_LAUNCH("ncf_ids_div");
  return NCF_OK;
}
