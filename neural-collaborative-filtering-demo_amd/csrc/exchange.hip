// The row-sharded training step's exchange kernels (multi-GPU data parallelism, SURVEY §8(e);
// the protocol and the RCCL collectives are in distributed.py).  owner(id) = id mod W, local row
// = id div W, R = ceil(rows / W) local rows per shard.
//
// Requester side (ncf_shard_plan): the batch ids are re-keyed as key = owner * R + local row and
// deduplicated with the radix dedup of dedup.hip.  Sorted keys are grouped by owner (ascending
// local row inside an owner), so the compact order of the unique rows IS the send order: the
// all-to-all send buffer is written straight from the unique keys (destination-major, users then
// items per destination), and a row's compact index c maps to its send position spos[c] without
// any permutation pass.  The dedup's segment structure stays in the workspace for the backward's
// segment reduce (ncf_embedding_bwd_reduce), exactly as on one GPU.
//
// Owner side: the received local rows are deduplicated WITHOUT a sort.  Every requester sent
// unique rows, so a row occurs at most once per source rank: a per-row token claim (atomicExch of
// the step's token into mark[row]) elects one claimer that appends the row to the unique list;
// a second pass records pos[u][s] = the position of row u's entry from source s.  The unique
// list's order is whatever the claims produce (nothing depends on it), the gradient sum of row u
// runs over s = 0..W-1 in rank order: deterministic and independent of scheduling.
//
// Reference: the single-process EBC lookup + dense-gradient Adam (src/model/architecture.py:
// 286-287, src/model/trainer.py:285); torchrec's sharded EBC is the reference's scale-out path.
#include "ncf_common.h"

namespace {

// ---- requester: plan ----------------------------------------------------------------------
__global__ void k_shard_keys(const int64_t* __restrict__ uid, const int64_t* __restrict__ iid,
                             int64_t n, int W, int64_t R0, int64_t R1, int64_t rows0,
                             int64_t rows1, int64_t* __restrict__ k0, int64_t* __restrict__ k1,
                             int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t u = uid[i], v = iid[i];
  if (u < 0 || u >= rows0) { atomicOr(err, 1); u = 0; }
  if (v < 0 || v >= rows1) { atomicOr(err, 2); v = 0; }
  k0[i] = (u % W) * R0 + u / W;
  k1[i] = (v % W) * R1 + v / W;
}

// first index of uniq[0 .. n) with key >= x (uniq ascending)
__device__ __forceinline__ int32_t lower_bound64(const int64_t* __restrict__ a, int32_t n, int64_t x) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// one block: bounds[k][o] = first unique key of owner o (o = 0..W), counts[o][k], and the
// destination offsets off[o] = sum_{d < o} (counts[d][0] + counts[d][1])  (off[W] = total)
__global__ void k_shard_bounds(const int64_t* __restrict__ uq0, const int64_t* __restrict__ uq1,
                               const uint32_t* __restrict__ num_unique, int W, int64_t R0,
                               int64_t R1, int32_t* __restrict__ bounds,
                               int64_t* __restrict__ counts) {
  __shared__ int32_t b[2][NCF_SHARD_MAX_WORLD + 1];
  const int t = threadIdx.x;
  if (t < 2 * (W + 1)) {
    const int k = t / (W + 1), o = t % (W + 1);
    const int32_t n = (int32_t)num_unique[k];
    b[k][o] = o == W ? n : lower_bound64(k ? uq1 : uq0, n, (int64_t)o * (k ? R1 : R0));
  }
  __syncthreads();
  if (t == 0) {
    int32_t off = 0;
    for (int o = 0; o < W; ++o) {
      const int32_t c0 = b[0][o + 1] - b[0][o], c1 = b[1][o + 1] - b[1][o];
      counts[2 * o] = c0;
      counts[2 * o + 1] = c1;
      bounds[2 * (W + 1) + o] = off;   // off[o]
      off += c0 + c1;
    }
    bounds[2 * (W + 1) + W] = off;
  }
  if (t < 2 * (W + 1)) bounds[t] = b[t / (W + 1)][t % (W + 1)];
}

// send[spos] = local row of unique key c, spos[c] = its position (destination-major layout)
__global__ void k_shard_send(const int64_t* __restrict__ uq0, const int64_t* __restrict__ uq1,
                             const uint32_t* __restrict__ num_unique, int W, int64_t R0,
                             int64_t R1, const int32_t* __restrict__ bounds,
                             int32_t* __restrict__ send, int32_t* __restrict__ spos0,
                             int32_t* __restrict__ spos1) {
  const int k = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= (int64_t)num_unique[k]) return;
  const int64_t key = (k ? uq1 : uq0)[c];
  const int64_t R = k ? R1 : R0;
  const int o = (int)(key / R);
  const int32_t* b0 = bounds;
  const int32_t* b1 = bounds + (W + 1);
  const int32_t* off = bounds + 2 * (W + 1);
  const int32_t pos = off[o] + (k ? (b0[o + 1] - b0[o]) + (int32_t)c - b1[o] : (int32_t)c - b0[o]);
  send[pos] = (int32_t)(key - (int64_t)o * R);
  (k ? spos1 : spos0)[c] = pos;
}

// rows?[r] = spos?[inv?[r]]: row r's send position (its received row, read in place by the
// forward gather); the int64 copies of spos are the embedding backward's table-row ids
__global__ void k_shard_rowpos(const int64_t* __restrict__ inv0, const int64_t* __restrict__ inv1,
                               const int32_t* __restrict__ spos0, const int32_t* __restrict__ spos1,
                               const uint32_t* __restrict__ num_unique, int64_t n,
                               int64_t* __restrict__ sp64_0, int64_t* __restrict__ sp64_1,
                               int64_t* __restrict__ rows0, int64_t* __restrict__ rows1) {
  const int k = blockIdx.y;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t* sp = k ? spos1 : spos0;
  if (r < n) (k ? rows1 : rows0)[r] = (int64_t)sp[(k ? inv1 : inv0)[r]];
  if (r < (int64_t)num_unique[k]) (k ? sp64_1 : sp64_0)[r] = (int64_t)sp[r];
}

// ---- owner ---------------------------------------------------------------------------------
// source rank and kind of received entry j
__device__ __forceinline__ void recv_src(const ncf_shard_recv& L, int32_t j, int& s, int& kind) {
  int lo = 0, hi = L.world - 1;   // last s with start[s] <= j
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.start[mid] <= j) lo = mid; else hi = mid - 1;
  }
  s = lo;
  kind = j < L.start[s] + L.n0[s] ? 0 : 1;
}

// One claimer per row (token exchange); the claimers of a wave take consecutive unique slots
// with ONE atomicAdd per kind and wave (a per-thread atomic on the shared counter serialises
// ~20K adds on one address).
__global__ __launch_bounds__(256) void k_owner_claim(
    const int32_t* __restrict__ recv, const ncf_shard_recv L, int32_t token,
    int32_t* __restrict__ mark0, int32_t* __restrict__ mark1, int32_t* __restrict__ uidx0,
    int32_t* __restrict__ uidx1, int64_t rows0, int64_t rows1, int64_t* __restrict__ uq0,
    int64_t* __restrict__ uq1, uint32_t* __restrict__ count, int32_t* __restrict__ pos0,
    int32_t* __restrict__ pos1, int* __restrict__ err) {
  const int32_t j = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  const int lane = threadIdx.x & 63;
  bool claim = false;
  int s = 0, k = 0;
  int32_t row = 0;
  if (j < L.start[L.world]) {
    recv_src(L, j, s, k);
    row = recv[j];
    if (row < 0 || row >= (k ? rows1 : rows0)) {
      atomicOr(err, 4);
    } else {
      claim = atomicExch((k ? mark1 : mark0) + row, token) != token;
    }
  }
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const uint64_t m = __ballot(claim && k == kk);
    if (!m) continue;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count + kk, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (claim && k == kk) {
      const uint32_t u = base + (uint32_t)__popcll(m & lt);
      (kk ? uidx1 : uidx0)[row] = (int32_t)u;
      (kk ? uq1 : uq0)[u] = row;
      int32_t* p = (kk ? pos1 : pos0) + (int64_t)u * L.world;
      for (int x = 0; x < L.world; ++x) p[x] = -1;
    }
  }
}

__global__ void k_owner_pos(const int32_t* __restrict__ recv, const ncf_shard_recv L,
                            const int32_t* __restrict__ uidx0, const int32_t* __restrict__ uidx1,
                            int64_t rows0, int64_t rows1, int32_t* __restrict__ pos0,
                            int32_t* __restrict__ pos1) {
  const int32_t j = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (j >= L.start[L.world]) return;
  int s, k;
  recv_src(L, j, s, k);
  const int32_t row = recv[j];
  if (row < 0 || row >= (k ? rows1 : rows0)) return;
  const int32_t u = (k ? uidx1 : uidx0)[row];
  (k ? pos1 : pos0)[(int64_t)u * L.world + s] = j;
}

// out[j] = (t?0[row] | t?1[row]) of the entry's kind; 16 lanes x float4 per D=64 half-row
template <int D>
__global__ void k_owner_gather(const int32_t* __restrict__ recv, const ncf_shard_recv L,
                               const float* __restrict__ t00, const float* __restrict__ t01,
                               int64_t rows0, const float* __restrict__ t10,
                               const float* __restrict__ t11, int64_t rows1,
                               float* __restrict__ out) {
  constexpr int LN = D / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t j = (int32_t)(t / LN);
  const int sub = (int)(t % LN);
  if (j >= L.start[L.world]) return;
  int s, k;
  recv_src(L, j, s, k);
  int64_t row = recv[j];
  if (row < 0 || row >= (k ? rows1 : rows0)) row = 0;   // flagged by k_owner_claim
  const float* a = k ? t10 : t00;
  const float* b = k ? t11 : t01;
  st4(out + (int64_t)j * 2 * D + sub * 4, ld4(a + row * D + sub * 4));
  st4(out + (int64_t)j * 2 * D + D + sub * 4, ld4(b + row * D + sub * 4));
}

// g?0[u] / g?1[u] = sum over sources s (rank order) of got[pos[u][s]] halves
template <int D>
__global__ void k_owner_gradsum(const float* __restrict__ got, const int32_t* __restrict__ pos0,
                                const int32_t* __restrict__ pos1,
                                const uint32_t* __restrict__ count, int W,
                                float* __restrict__ g00, float* __restrict__ g01,
                                float* __restrict__ g10, float* __restrict__ g11) {
  constexpr int LN = D / 4;
  const int k = blockIdx.y;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t u = t / LN;
  const int sub = (int)(t % LN);
  if (u >= (int64_t)count[k]) return;
  const int32_t* p = (k ? pos1 : pos0) + u * W;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  for (int s = 0; s < W; ++s) {
    const int32_t j = p[s];
    if (j < 0) continue;
    const float4 x = ld4(got + (int64_t)j * 2 * D + sub * 4);
    const float4 y = ld4(got + (int64_t)j * 2 * D + D + sub * 4);
    a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
  }
  st4((k ? g10 : g00) + u * D + sub * 4, a);
  st4((k ? g11 : g01) + u * D + sub * 4, b);
}

// ---- requester: rows in / gradients out ------------------------------------------------------
// dir 0: mini?[c] = back[spos?[c]] halves;  dir 1: buf[spos?[c]] = (g?0[c] | g?1[c])
template <int D>
__global__ void k_shard_rows(float* __restrict__ buf, const int32_t* __restrict__ spos0,
                             const int32_t* __restrict__ spos1,
                             const uint32_t* __restrict__ num_unique, float* __restrict__ m00,
                             float* __restrict__ m01, float* __restrict__ m10,
                             float* __restrict__ m11, int dir) {
  constexpr int LN = D / 4;
  const int k = blockIdx.y;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = t / LN;
  const int sub = (int)(t % LN);
  if (c >= (int64_t)num_unique[k]) return;
  float* r = buf + (int64_t)(k ? spos1 : spos0)[c] * 2 * D + sub * 4;
  float* a = (k ? m10 : m00) + c * D + sub * 4;
  float* b = (k ? m11 : m01) + c * D + sub * 4;
  if (dir == 0) {
    st4(a, ld4(r));
    st4(b, ld4(r + D));
  } else {
    st4(r, ld4(a));
    st4(r + D, ld4(b));
  }
}

bool dim_ok(int64_t dim) { return dim == 16 || dim == 32 || dim == 64 || dim == 128 || dim == 256; }

#define NCF_EX_DISPATCH(D, KERNEL, GRID, BLOCK, ST, ...)                                   \
  switch (D) {                                                                             \
    case 16: hipLaunchKernelGGL(KERNEL<16>, GRID, BLOCK, 0, ST, __VA_ARGS__); break;       \
    case 32: hipLaunchKernelGGL(KERNEL<32>, GRID, BLOCK, 0, ST, __VA_ARGS__); break;       \
    case 64: hipLaunchKernelGGL(KERNEL<64>, GRID, BLOCK, 0, ST, __VA_ARGS__); break;       \
    case 128: hipLaunchKernelGGL(KERNEL<128>, GRID, BLOCK, 0, ST, __VA_ARGS__); break;     \
    default: hipLaunchKernelGGL(KERNEL<256>, GRID, BLOCK, 0, ST, __VA_ARGS__); break;      \
  }

bool layout_ok(const ncf_shard_recv* L) {
  if (!L || L->world < 1 || L->world > NCF_SHARD_MAX_WORLD || L->start[0] != 0) return false;
  for (int s = 0; s < L->world; ++s)
    if (L->n0[s] < 0 || L->start[s + 1] < L->start[s] + L->n0[s]) return false;
  return true;
}

}  // namespace

extern "C" int ncf_shard_plan(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                              int world, int64_t num_users, int64_t num_items, int64_t dim,
                              const ncf_shard_plan_out* o, void* workspace,
                              int64_t workspace_bytes, int* err_flag, void* stream) {
  NCF_CHECK_ARG(o && n >= 0 && n < (1ll << 30) && world >= 1 && world <= NCF_SHARD_MAX_WORLD &&
                    num_users >= 1 && num_items >= 1 && dim_ok(dim) && err_flag,
                "ncf_shard_plan: bad args");
  NCF_CHECK_ARG(o->keys0 && o->keys1 && o->uniq0 && o->uniq1 && o->num_unique && o->inv0 &&
                    o->inv1 && o->counts && o->send && o->spos0 && o->spos1 && o->bounds,
                "ncf_shard_plan: null output");
  hipStream_t st = (hipStream_t)stream;
  const int64_t R0 = (num_users + world - 1) / world, R1 = (num_items + world - 1) / world;
  if (n > 0) {
    hipLaunchKernelGGL(k_shard_keys, dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, user_ids, item_ids,
                       n, world, R0, R1, num_users, num_items, o->keys0, o->keys1, err_flag);
    NCF_CHECK_LAUNCH("ncf_shard_plan(keys)");
  }
  int rc = ncf_dedup_ids2(o->keys0, n, R0 * world, o->keys1, n, R1 * world, dim, o->uniq0,
                          o->uniq1, nullptr, nullptr, o->num_unique, workspace, workspace_bytes,
                          stream);
  if (rc) return rc;
  rc = ncf_dedup_inverse(n, n, R0 * world, R1 * world, dim, o->inv0, o->inv1, workspace,
                         workspace_bytes, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_shard_bounds, dim3(1), dim3(2 * NCF_SHARD_MAX_WORLD + 2), 0, st, o->uniq0,
                     o->uniq1, o->num_unique, world, R0, R1, o->bounds, o->counts);
  NCF_CHECK_LAUNCH("ncf_shard_plan(bounds)");
  if (n > 0) {
    hipLaunchKernelGGL(k_shard_send, dim3(ncf_cdiv(n, 256), 2), dim3(256), 0, st, o->uniq0,
                       o->uniq1, o->num_unique, world, R0, R1, o->bounds, o->send, o->spos0,
                       o->spos1);
    NCF_CHECK_LAUNCH("ncf_shard_plan(send)");
    if (o->spos64_0 && o->spos64_1 && o->rows0 && o->rows1) {
      hipLaunchKernelGGL(k_shard_rowpos, dim3(ncf_cdiv(n, 256), 2), dim3(256), 0, st, o->inv0,
                         o->inv1, o->spos0, o->spos1, o->num_unique, n, o->spos64_0, o->spos64_1,
                         o->rows0, o->rows1);
      NCF_CHECK_LAUNCH("ncf_shard_plan(rowpos)");
    }
  }
  return NCF_OK;
}

extern "C" int ncf_shard_owner_prepare(const int32_t* recv, const ncf_shard_recv* layout,
                                       int32_t token, int32_t* mark0, int32_t* mark1,
                                       int32_t* uidx0, int32_t* uidx1, int64_t rows0,
                                       int64_t rows1, int64_t* uniq0, int64_t* uniq1,
                                       uint32_t* count, int32_t* pos0, int32_t* pos1,
                                       int* err_flag, void* stream) {
  NCF_CHECK_ARG(layout_ok(layout), "ncf_shard_owner_prepare: bad receive layout");
  NCF_CHECK_ARG(token > 0 && mark0 && mark1 && uidx0 && uidx1 && uniq0 && uniq1 && count &&
                    pos0 && pos1 && err_flag && rows0 >= 1 && rows1 >= 1,
                "ncf_shard_owner_prepare: bad args");
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(count, 0, 2 * sizeof(uint32_t), st);
  const int32_t total = layout->start[layout->world];
  if (total == 0) return NCF_OK;
  NCF_CHECK_ARG(recv != nullptr, "ncf_shard_owner_prepare: null recv");
  hipLaunchKernelGGL(k_owner_claim, dim3(ncf_cdiv(total, 256)), dim3(256), 0, st, recv, *layout,
                     token, mark0, mark1, uidx0, uidx1, rows0, rows1, uniq0, uniq1, count, pos0,
                     pos1, err_flag);
  NCF_CHECK_LAUNCH("ncf_shard_owner_prepare(claim)");
  hipLaunchKernelGGL(k_owner_pos, dim3(ncf_cdiv(total, 256)), dim3(256), 0, st, recv, *layout,
                     uidx0, uidx1, rows0, rows1, pos0, pos1);
  NCF_CHECK_LAUNCH("ncf_shard_owner_prepare(pos)");
  return NCF_OK;
}

extern "C" int ncf_shard_owner_gather(const int32_t* recv, const ncf_shard_recv* layout,
                                      const float* t00, const float* t01, int64_t rows0,
                                      const float* t10, const float* t11, int64_t rows1,
                                      int64_t dim, float* out, void* stream) {
  NCF_CHECK_ARG(layout_ok(layout) && dim_ok(dim), "ncf_shard_owner_gather: bad args");
  const int32_t total = layout->start[layout->world];
  if (total == 0) return NCF_OK;
  NCF_CHECK_ARG(recv && t00 && t01 && t10 && t11 && out, "ncf_shard_owner_gather: null pointer");
  const int64_t threads = (int64_t)total * (dim / 4);
  NCF_EX_DISPATCH(dim, k_owner_gather, dim3(ncf_cdiv(threads, 256)), dim3(256), (hipStream_t)stream,
                  recv, *layout, t00, t01, rows0, t10, t11, rows1, out);
  NCF_CHECK_LAUNCH("ncf_shard_owner_gather");
  return NCF_OK;
}

extern "C" int ncf_shard_owner_gradsum(const float* got, const int32_t* pos0, const int32_t* pos1,
                                       const uint32_t* count, int64_t max_unique, int world,
                                       int64_t dim, float* g00, float* g01, float* g10, float* g11,
                                       void* stream) {
  NCF_CHECK_ARG(world >= 1 && world <= NCF_SHARD_MAX_WORLD && dim_ok(dim) && max_unique >= 0,
                "ncf_shard_owner_gradsum: bad args");
  if (max_unique == 0) return NCF_OK;
  NCF_CHECK_ARG(got && pos0 && pos1 && count && g00 && g01 && g10 && g11,
                "ncf_shard_owner_gradsum: null pointer");
  const int64_t threads = max_unique * (dim / 4);
  NCF_EX_DISPATCH(dim, k_owner_gradsum, dim3(ncf_cdiv(threads, 256), 2), dim3(256),
                  (hipStream_t)stream, got, pos0, pos1, count, world, g00, g01, g10, g11);
  NCF_CHECK_LAUNCH("ncf_shard_owner_gradsum");
  return NCF_OK;
}

extern "C" int ncf_shard_rows(float* buf, const int32_t* spos0, const int32_t* spos1,
                              const uint32_t* num_unique, int64_t max_n, int64_t dim, float* m00,
                              float* m01, float* m10, float* m11, int dir, void* stream) {
  NCF_CHECK_ARG(dim_ok(dim) && max_n >= 0 && (dir == 0 || dir == 1), "ncf_shard_rows: bad args");
  if (max_n == 0) return NCF_OK;
  NCF_CHECK_ARG(buf && spos0 && spos1 && num_unique && m00 && m01 && m10 && m11,
                "ncf_shard_rows: null pointer");
  const int64_t threads = max_n * (dim / 4);
  NCF_EX_DISPATCH(dim, k_shard_rows, dim3(ncf_cdiv(threads, 256), 2), dim3(256), (hipStream_t)stream,
                  buf, spos0, spos1, num_unique, m00, m01, m10, m11, dir);
  NCF_CHECK_LAUNCH("ncf_shard_rows");
  return NCF_OK;
}
