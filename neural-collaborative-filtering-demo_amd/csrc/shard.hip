// Row sharding over W ranks (multi-GPU data parallelism): owner(id) = id mod W,
// local row = id div W.  Pack / unpack kernels around the RCCL all-to-alls of
// distributed.py (the collectives themselves run in torch.distributed): owner bucketing of the
// deduplicated batch ids (one stable 8-bit radix pass), shard row gathers, permutations, and the
// owner-side fixed-order segment sums of the received gradient rows.
//
// Reference: the single-process EBC lookup + dense-gradient Adam (src/model/architecture.py:
// 286-287, src/model/trainer.py:285); torchrec's sharded EBC is the reference's intended scale-out.
#include "segments.h"

using namespace ncf_seg;

namespace {

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

// after one stable pass: send_ids[j] = uniq[perm[j]] div W, counts[kind][d] from the scanned
// histogram
__global__ void k_owner_finish(const int64_t* __restrict__ uniq0, const int64_t* __restrict__ uniq1,
                               const uint32_t* __restrict__ count, const uint32_t* __restrict__ sv0,
                               const uint32_t* __restrict__ sv1, int64_t n,
                               const uint32_t* __restrict__ offs, int nb, int W,
                               int64_t* __restrict__ send0, int64_t* __restrict__ send1,
                               int32_t* __restrict__ perm0, int32_t* __restrict__ perm1,
                               int64_t* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the owner's LOCAL row (id div W) is what travels: owners index their shard directly
  if (i < (int64_t)count[0]) { perm0[i] = (int32_t)sv0[i]; send0[i] = uniq0[sv0[i]] / W; }
  if (i < (int64_t)count[1]) { perm1[i] = (int32_t)sv1[i]; send1[i] = uniq1[sv1[i]] / W; }
  if (blockIdx.x == 0 && threadIdx.x < 2 * W) {
    const int kind = threadIdx.x / W, d = threadIdx.x % W;
    const uint32_t* o = offs + (int64_t)kind * 256 * nb;
    counts[kind * W + d] = (int64_t)(o[(int64_t)(d + 1) * nb] - o[(int64_t)d * nb]);
  }
  (void)n;
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

}  // namespace

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
  sorted_bufs(w, sort_passes(rows0, rows1), &k0, &v0, &k1, &v1);
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
