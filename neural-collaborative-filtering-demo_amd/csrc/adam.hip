// Fused Adam for the AdvancedNCF parameters — torch.optim.Adam(model.parameters(), lr,
// weight_decay) semantics exactly as the reference trainer constructs it
// (src/model/trainer.py:71-75; step at :285):
//   g += wd * p                    (coupled L2, every element, every step)
//   m  = m + (1-b1) * (g - m)      (exp_avg.lerp_)
//   v  = v * b2 + (1-b2) * g * g   (exp_avg_sq.mul_.addcmul_)
//   p += -step_size * m / (sqrt(v) / sqrt(1-b2^t) + eps),   step_size = lr / (1-b1^t)
// Scalars are computed on the host in double and rounded to fp32, as torch does.
//
// Embedding tables are updated DENSE-EXACT: the reference's dense [rows, D] gradient is zero on
// untouched rows, but weight decay makes every row move every step, so every
// element of every table is streamed.  Touched rows take their gradient from the compact buffer
// written by ncf_embedding_bwd through the slot map (slot[row] = compact index or -1): the
// per-step traffic is exactly p, m, v read+write (24 B/element) + 4 B/row slot + the touched rows.
// HBM-bound: float4 per lane, grid-stride over the table.
#include "ncf_common.h"
#include "adam_math.h"

using namespace ncf_adam;

namespace {


template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_adam_table(float* __restrict__ p, float* __restrict__ m,
                                                    float* __restrict__ v, int64_t rows,
                                                    const int32_t* __restrict__ slot,
                                                    const float* __restrict__ G, AdamScalars s) {
  const int64_t n4 = rows * (D / 4);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n4;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / (D / 4);
    const int col = (int)(e % (D / 4)) * 4;
    const int32_t sl = slot ? slot[row] : -1;
    float4 pp = ldp4<BF>(p, e * 4), mm = ld4(m + e * 4), vv = ld4(v + e * 4);
    if (sl >= 0) {
      adam4(pp, mm, vv, ld4(G + (int64_t)sl * D + col), s);
    } else {   // no gradient row this step: the zero-gradient form (as the deferred replay)
      adam0(pp.x, mm.x, vv.x, s.ra, s.rb, s);
      adam0(pp.y, mm.y, vv.y, s.ra, s.rb, s);
      adam0(pp.z, mm.z, vv.z, s.ra, s.rb, s);
      adam0(pp.w, mm.w, vv.w, s.ra, s.rb, s);
    }
    stp4<BF>(p, e * 4, pp);
    st4(m + e * 4, mm);
    st4(v + e * 4, vv);
  }
}

__global__ __launch_bounds__(256) void k_adam_flat(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, AdamScalars s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam1(pp, mm, vv, g[i], s);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

// A table with a dense [rows, D] gradient (gradient accumulation and the other dense-.grad
// cases of the optimizer hook): an element whose gradient is exactly zero takes the
// zero-gradient form, as the row-sparse schedules step the rows that got no gradient (a touched
// row's gradient is never exactly zero in practice: it comes through the LayerNorm backward).
__global__ __launch_bounds__(256) void k_adam_table_dense_grad(float* __restrict__ p,
                                                               const float* __restrict__ g,
                                                               float* __restrict__ m,
                                                               float* __restrict__ v, int64_t n,
                                                               AdamScalars s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    const float gg = g[i];
    if (gg == 0.0f) adam0(pp, mm, vv, s.ra, s.rb, s);
    else adam1(pp, mm, vv, gg, s);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

// dense[uniq[c]] = G[c] for c < num_unique[kind]  (materialise a dense table gradient)
template <int D>
__global__ void k_scatter_compact(float* __restrict__ dense, const int64_t* __restrict__ uniq,
                                  const uint32_t* __restrict__ num_unique, int kind,
                                  const float* __restrict__ G, int64_t max_n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = t / (D / 4);
  const int col = (int)(t % (D / 4)) * 4;
  if (c >= max_n || c >= (int64_t)num_unique[kind]) return;
  st4(dense + uniq[c] * D + col, ld4(G + c * D + col));
}

// ---- deferred dense-exact schedule -------------------------------------------------------
// A row that receives no gradient at step s still takes the step with g = 0 (weight decay only).
// Instead of streaming every untouched row every step, rows carry stamp[row] = the last step
// their (p, m, v) reflect; before a row is READ it is caught up by replaying the missing
// zero-gradient steps s = stamp+1 .. target with that step's scalars (step table, 4 floats per
// step: [4s] = -lr/(1-b1^s), [4s+1] = 1/sqrt(1-b2^s) for the gradient step adam1, [4s+2] / [4s+3]
// = ra / rb for the zero-gradient step adam0), element by element, with the very same adam0
// arithmetic as the dense sweep's untouched rows.
// Results are bit-identical to the dense sweep; the cost moves from HBM traffic to VALU work.
struct TablePtrs {
  float *p0, *m0, *v0, *p1, *m1, *v1;  // two tables sharing the row index space (GMF + MLP)
  const float *G0, *G1;                 // compact gradients (apply only)
};

// Replay layout: lane = column.  One row (of both tables of a pair) per wave when D >= 64
// (EPL = D/64 columns per lane, stride 64), 64/D rows per wave when D < 64.  With one row per
// wave the replay bounds (from, to) are wave-uniform: the step loop is scalar, the per-step
// scalars come through the scalar cache, and no lane idles on another row's longer catch-up.
template <int D>
struct Replay {
  static constexpr int LPR = D < 64 ? D : 64;   // lanes per row
  static constexpr int EPL = D / LPR;           // columns per lane
};

// The replay of zero-gradient steps from+1 .. to on EPL columns of one (pair of) table row(s).
// With wave-uniform bounds (one row per wave) the per-step scalars are scalar loads; they are
// fetched 8 steps (16 floats) at a time, one chunk AHEAD of the steps that use them, so the
// scalar-load latency hides behind 8 steps of VALU work instead of stalling every step (the
// step table is padded >= 4096 steps past any target, deferred.py _ensure).  Same adam1 calls in
// the same order: results are bit-identical to the step-by-step loop.
template <int EPL, bool PAIR, bool BF = false>
__device__ __forceinline__ void replay_uniform(float* p0, float* m0, float* v0, float* p1,
                                               float* m1, float* v1, int32_t from, int32_t to,
                                               const float* __restrict__ table,
                                               const AdamScalars& s) {
  constexpr int C = 8;                 // steps per chunk
  int32_t q = from + 1;
  float sc[2 * C];
#pragma unroll
  for (int k = 0; k < C; ++k) {
    sc[2 * k] = table[4 * (q + k) + 2];
    sc[2 * k + 1] = table[4 * (q + k) + 3];
  }
  while (q + C - 1 <= to) {
    float nx[2 * C];
#pragma unroll
    for (int k = 0; k < C; ++k) {
      nx[2 * k] = table[4 * (q + C + k) + 2];
      nx[2 * k + 1] = table[4 * (q + C + k) + 3];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of this chunk's steps
#pragma unroll
    for (int k = 0; k < C; ++k) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        adam0(p0[j], m0[j], v0[j], sc[2 * k], sc[2 * k + 1], s);
        if (BF) p0[j] = ncf_round_bf16(p0[j]);   // bf16 tables: stored (rounded) every step
        if (PAIR) adam0(p1[j], m1[j], v1[j], sc[2 * k], sc[2 * k + 1], s);
        if (PAIR && BF) p1[j] = ncf_round_bf16(p1[j]);
      }
    }
#pragma unroll
    for (int k = 0; k < 2 * C; ++k) sc[k] = nx[k];
    q += C;
  }
#pragma unroll
  for (int k = 0; k < C - 1; ++k) {    // the last to - q + 1 < C steps
    if (q + k > to) break;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      adam0(p0[j], m0[j], v0[j], sc[2 * k], sc[2 * k + 1], s);
      if (BF) p0[j] = ncf_round_bf16(p0[j]);
      if (PAIR) adam0(p1[j], m1[j], v1[j], sc[2 * k], sc[2 * k + 1], s);
      if (PAIR && BF) p1[j] = ncf_round_bf16(p1[j]);
    }
  }
}

template <int D, bool BF = false>
__device__ __forceinline__ void catch_up_row(const TablePtrs& t, int64_t row, int sub, int32_t from,
                                             int32_t to, const float* __restrict__ table,
                                             const AdamScalars& s) {
  constexpr int EPL = Replay<D>::EPL, LPR = Replay<D>::LPR;
  if (Replay<D>::LPR == 64) {   // the whole wave holds this row: make the bounds scalar
    from = __builtin_amdgcn_readfirstlane(from);
    to = __builtin_amdgcn_readfirstlane(to);
  }
  if (from >= to) return;
  const int64_t o = row * D + sub;
  float p0[EPL], m0[EPL], v0[EPL], p1[EPL], m1[EPL], v1[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    p0[j] = ldp<BF>(t.p0, o + j * LPR); m0[j] = t.m0[o + j * LPR]; v0[j] = t.v0[o + j * LPR];
  }
  if (t.p1) {
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      p1[j] = ldp<BF>(t.p1, o + j * LPR); m1[j] = t.m1[o + j * LPR]; v1[j] = t.v1[o + j * LPR];
    }
    if (Replay<D>::LPR == 64) {
      replay_uniform<EPL, true, BF>(p0, m0, v0, p1, m1, v1, from, to, table, s);
    } else {
#pragma unroll 2
      for (int32_t q = from + 1; q <= to; ++q) {
        const float ra = table[4 * q + 2], rb = table[4 * q + 3];
#pragma unroll
        for (int j = 0; j < EPL; ++j) {
          adam0(p0[j], m0[j], v0[j], ra, rb, s);
          adam0(p1[j], m1[j], v1[j], ra, rb, s);
          if (BF) { p0[j] = ncf_round_bf16(p0[j]); p1[j] = ncf_round_bf16(p1[j]); }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      stp<BF>(t.p1, o + j * LPR, p1[j]); t.m1[o + j * LPR] = m1[j]; t.v1[o + j * LPR] = v1[j];
    }
  } else if (Replay<D>::LPR == 64) {
    replay_uniform<EPL, false, BF>(p0, m0, v0, p1, m1, v1, from, to, table, s);
  } else {
#pragma unroll 2
    for (int32_t q = from + 1; q <= to; ++q) {
      const float ra = table[4 * q + 2], rb = table[4 * q + 3];
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        adam0(p0[j], m0[j], v0[j], ra, rb, s);
        if (BF) p0[j] = ncf_round_bf16(p0[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    stp<BF>(t.p0, o + j * LPR, p0[j]); t.m0[o + j * LPR] = m0[j]; t.v0[o + j * LPR] = v0[j];
  }
}

// rows listed in ids[0 .. count[kind]) (unique), caught up to `target`
template <int D>
__global__ __launch_bounds__(256) void k_adam_catchup(TablePtrs t, const int64_t* __restrict__ ids,
                                                      const uint32_t* __restrict__ count, int kind,
                                                      int64_t max_n, int32_t* __restrict__ stamp,
                                                      int32_t target, const float* __restrict__ table,
                                                      AdamScalars s,
                                                      const ncf_step_clock* __restrict__ clock) {
  constexpr int L = Replay<D>::LPR;   // lanes per row
  const int64_t tt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = tt / L;
  const int sub = (int)(tt % L);
  const int64_t cnt = count ? (int64_t)count[kind] : max_n;
  if (c >= max_n || c >= cnt) return;
  if (clock) target += clock->t;
  const int64_t row = ids[c];
  const int32_t from = stamp[row];
  catch_up_row<D>(t, row, sub, from, target, table, s);
  if (sub == 0 && from < target) stamp[row] = target;
}

// every row of the table caught up to `target` (materialise)
template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_adam_sweep(TablePtrs t, int64_t row0, int64_t rows,
                                                    int32_t* __restrict__ stamp, int32_t target,
                                                    const float* __restrict__ table, AdamScalars s) {
  constexpr int L = Replay<D>::LPR;   // lanes per row
  const int64_t n = rows * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = row0 + e / L;
    const int sub = (int)(e % L);
    const int32_t from = stamp[row];
    catch_up_row<D, BF>(t, row, sub, from, target, table, s);
    // all L lanes of the row read stamp before this store: they share one wave-instruction
    if (sub == 0 && from < target) stamp[row] = target;
  }
}

// step `step` applied to the touched rows (already current through step-1) with their gradient
template <int D>
__global__ __launch_bounds__(256) void k_adam_apply(TablePtrs t, const int64_t* __restrict__ ids,
                                                    const uint32_t* __restrict__ count, int kind,
                                                    int64_t max_n, int32_t* __restrict__ stamp,
                                                    int32_t step, const float* __restrict__ table,
                                                    AdamScalars s,
                                                    const ncf_step_clock* __restrict__ clock) {
  constexpr int L = D / 4;
  const int64_t tt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = tt / L;
  const int sub = (int)(tt % L);
  const int64_t cnt = count ? (int64_t)count[kind] : max_n;
  if (c >= max_n || c >= cnt) return;
  if (clock) step += clock->t;
  const int64_t row = ids[c];
  const int64_t o = row * D + sub * 4;
  const float ns = table[4 * step], bc = table[4 * step + 1];
  float4 p0 = ld4(t.p0 + o), m0 = ld4(t.m0 + o), v0 = ld4(t.v0 + o);
  adam4(p0, m0, v0, ld4(t.G0 + c * D + sub * 4), ns, bc, s);
  st4(t.p0 + o, p0); st4(t.m0 + o, m0); st4(t.v0 + o, v0);
  if (t.p1) {
    float4 p1 = ld4(t.p1 + o), m1 = ld4(t.m1 + o), v1 = ld4(t.v1 + o);
    adam4(p1, m1, v1, ld4(t.G1 + c * D + sub * 4), ns, bc, s);
    st4(t.p1 + o, p1); st4(t.m1 + o, m1); st4(t.v1 + o, v1);
  }
  if (sub == 0) stamp[row] = step;
}

// rolling sweep of a captured step: closes step s = clock->t + step_rel, slice (s mod every)
template <int D>
__global__ __launch_bounds__(256) void k_adam_sweep_rolling(TablePtrs t, int64_t total_rows,
                                                            int64_t slice, int32_t every,
                                                            int32_t* __restrict__ stamp,
                                                            int32_t step_rel,
                                                            const ncf_step_clock* __restrict__ clock,
                                                            const float* __restrict__ table,
                                                            AdamScalars s) {
  constexpr int L = Replay<D>::LPR;   // lanes per row
  const int32_t target = clock->t + step_rel;
  const int64_t row0 = (int64_t)(target % every) * slice;
  const int64_t rows = max((int64_t)0, min(slice, total_rows - row0));
  const int64_t n = rows * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = row0 + e / L;
    const int sub = (int)(e % L);
    const int32_t from = stamp[row];
    catch_up_row<D>(t, row, sub, from, target, table, s);
    if (sub == 0 && from < target) stamp[row] = target;
  }
}

// flat Adam of step clock->t + step_rel with the step table's scalars
__global__ __launch_bounds__(256) void k_adam_flat_clock(float* __restrict__ p,
                                                         const float* __restrict__ g,
                                                         float* __restrict__ m,
                                                         float* __restrict__ v, int64_t n,
                                                         const float* __restrict__ table,
                                                         int32_t step_rel,
                                                         const ncf_step_clock* __restrict__ clock,
                                                         AdamScalars s) {
  const int32_t step = clock->t + step_rel;
  const float ns = table[4 * step], bc = table[4 * step + 1];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam1(pp, mm, vv, g[i], ns, bc, s);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

// ---- both id kinds per launch (blockIdx.y = kind)
struct PairArgs {
  TablePtrs t[2];
  const int64_t* ids[2];
  int32_t* stamp[2];
  int64_t rows[2];
  int bf;            // parameter rows are bf16 (host-side dispatch only)
};

template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_pairs_catchup(const PairArgs a, const uint32_t* __restrict__ count,
                                                       int64_t max_n, int32_t target_rel,
                                                       const ncf_step_clock* __restrict__ clock,
                                                       const float* __restrict__ table,
                                                       AdamScalars s, int lock) {
  constexpr int L = Replay<D>::LPR;   // lanes per row
  const int k = blockIdx.y;
  const int64_t tt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = tt / L;
  const int sub = (int)(tt % L);
  if (c >= max_n || c >= (int64_t)count[k]) return;
  const int32_t target = clock->t + target_rel;
  const int64_t row = a.ids[k][c];
  int32_t* stamp = a.stamp[k];
  const int32_t from = stamp[row];
  catch_up_row<D, BF>(a.t[k], row, sub, from, target, table, s);
  // lock: every listed row is marked in flight (current through target, its gradient step still
  // to come: the step's apply writes the plain stamp back); replays of other rows skip it
  if (sub == 0 && (lock || from < target)) stamp[row] = lock ? (target | NCF_STAMP_LOCK) : target;
}

// Claim form of the pair catch-up, with no dedup before it: one row-group of lanes per
// OCCURRENCE ids[k][0 .. n).  The first occurrence of a row to raise its stamp to `target`
// (atomicMax) replays it; every other occurrence sees the raised stamp and skips.  Exactly one
// replay per row, the same replay as k_pairs_catchup (bit-identical rows), so the id sort the
// backward needs can run on another stream beside the forward.  Locked rows (stamp = t |
// NCF_STAMP_LOCK) compare above any target and are left alone.  Out-of-range ids are skipped
// (the gather flags them).
template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_pairs_catchup_claim(const PairArgs a,
                                                             const int64_t* __restrict__ ids0,
                                                             const int64_t* __restrict__ ids1,
                                                             int64_t n, int32_t target_rel,
                                                             const ncf_step_clock* __restrict__ clock,
                                                             const float* __restrict__ table,
                                                             AdamScalars s) {
  constexpr int L = Replay<D>::LPR;   // lanes per row
  const int k = blockIdx.y;
  const int64_t tt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = tt / L;
  const int sub = (int)(tt % L);
  if (c >= n) return;
  const int64_t row = (k ? ids1 : ids0)[c];
  if (row < 0 || row >= a.rows[k]) return;
  const int32_t target = clock->t + target_rel;
  int32_t from = target;
  if (sub == 0) from = atomicMax(&a.stamp[k][row], target);
  from = __shfl(from, (int)(threadIdx.x & 63) - sub, 64);   // the claim of this row's lane group
  catch_up_row<D, BF>(a.t[k], row, sub, from, target, table, s);
}

template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_pairs_apply(const PairArgs a, const uint32_t* __restrict__ count,
                                                     int64_t max_n, int32_t step_rel,
                                                     const ncf_step_clock* __restrict__ clock,
                                                     const float* __restrict__ table, AdamScalars s) {
  constexpr int L = D / 4;
  const int k = blockIdx.y;
  const int64_t tt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = tt / L;
  const int sub = (int)(tt % L);
  if (c >= max_n || c >= (int64_t)count[k]) return;
  const int32_t step = clock->t + step_rel;
  const TablePtrs& t = a.t[k];
  const int64_t row = a.ids[k][c];
  const int64_t o = row * D + sub * 4;
  const float ns = table[4 * step], bc = table[4 * step + 1];
  // every load of both tables before any store: the compiler cannot know the two tables' rows
  // do not alias, and in program order the second table's loads would wait for the first
  // one's stores (two dependent HBM round trips per row instead of one)
  const bool two = t.p1 != nullptr;
  const int64_t og = c * D + sub * 4;
  float4 p0 = ldp4<BF>(t.p0, o), m0 = ld4(t.m0 + o), v0 = ld4(t.v0 + o), g0 = ld4(t.G0 + og);
  float4 p1 = {0.f, 0.f, 0.f, 0.f}, m1 = p1, v1 = p1, g1 = p1;
  if (two) {
    p1 = ldp4<BF>(t.p1, o); m1 = ld4(t.m1 + o); v1 = ld4(t.v1 + o); g1 = ld4(t.G1 + og);
  }
  adam4(p0, m0, v0, g0, ns, bc, s);
  if (two) adam4(p1, m1, v1, g1, ns, bc, s);
  stp4<BF>(t.p0, o, p0); st4(t.m0 + o, m0); st4(t.v0 + o, v0);
  if (two) { stp4<BF>(t.p1, o, p1); st4(t.m1 + o, m1); st4(t.v1 + o, v1); }
  if (sub == 0) a.stamp[k][row] = step;
}

// The owner side of the row-sharded step: the gradient of unique row c is the sum, in rank order,
// of the rows the W requesters sent for it (got[pos[c][s]]: [mf | mlp] halves of 2 D floats, -1
// where rank s did not touch the row) — summed here, in the order ncf_shard_owner_gradsum sums
// them (0 + x == x exactly: the same bits), then applied as k_pairs_apply does.
template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_pairs_apply_gsum(const PairArgs a, const uint32_t* __restrict__ count,
                                                          int64_t max_n, int32_t step_rel,
                                                          const ncf_step_clock* clock,
                                                          const float* __restrict__ table,
                                                          AdamScalars s,
                                                          const float* __restrict__ got,
                                                          const int32_t* __restrict__ pos0,
                                                          const int32_t* __restrict__ pos1, int W) {
  constexpr int L = D / 4;
  const int k = blockIdx.y;
  const int64_t tt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = tt / L;
  const int sub = (int)(tt % L);
  if (c >= max_n || c >= (int64_t)count[k]) return;
  const int32_t step = clock->t + step_rel;
  const TablePtrs& t = a.t[k];
  const int64_t row = a.ids[k][c];
  const int64_t o = row * D + sub * 4;
  const float ns = table[4 * step], bc = table[4 * step + 1];
  float4 p0 = ldp4<BF>(t.p0, o), m0 = ld4(t.m0 + o), v0 = ld4(t.v0 + o);
  float4 p1 = ldp4<BF>(t.p1, o), m1 = ld4(t.m1 + o), v1 = ld4(t.v1 + o);
  float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), g1 = g0;
  const int32_t* pp = (k ? pos1 : pos0) + c * W;
  for (int r = 0; r < W; ++r) {
    const int32_t j = pp[r];
    if (j < 0) continue;
    const float4 x = ld4(got + (int64_t)j * 2 * D + sub * 4);
    const float4 y = ld4(got + (int64_t)j * 2 * D + D + sub * 4);
    g0.x += x.x; g0.y += x.y; g0.z += x.z; g0.w += x.w;
    g1.x += y.x; g1.y += y.y; g1.z += y.z; g1.w += y.w;
  }
  adam4(p0, m0, v0, g0, ns, bc, s);
  adam4(p1, m1, v1, g1, ns, bc, s);
  stp4<BF>(t.p0, o, p0); st4(t.m0 + o, m0); st4(t.v0 + o, v0);
  stp4<BF>(t.p1, o, p1); st4(t.m1 + o, m1); st4(t.v1 + o, v1);
  if (sub == 0) a.stamp[k][row] = step;
}

// part `part` of `nparts` (consecutive row ranges) of the slice of step clock->t + step_rel
template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_pairs_sweep(const PairArgs a, int32_t every,
                                                     int32_t step_rel,
                                                     const ncf_step_clock* __restrict__ clock,
                                                     const float* __restrict__ table, AdamScalars s,
                                                     int part, int nparts) {
  constexpr int L = Replay<D>::LPR;   // lanes per row
  const int k = blockIdx.y;
  const int32_t target = clock->t + step_rel;
  const int64_t total = a.rows[k];
  const int64_t slice = (total + every - 1) / every;
  const int64_t s0 = (int64_t)(target % every) * slice;
  const int64_t srows = max((int64_t)0, min(slice, total - s0));
  const int64_t row0 = s0 + srows * part / nparts;
  const int64_t rows = s0 + srows * (part + 1) / nparts - row0;
  const int64_t n = rows * L;
  int32_t* stamp = a.stamp[k];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = row0 + e / L;
    const int sub = (int)(e % L);
    const int32_t from = stamp[row];
    catch_up_row<D, BF>(a.t[k], row, sub, from, target, table, s);
    if (sub == 0 && from < target) stamp[row] = target;
  }
}

__device__ __forceinline__ void clock_advance(ncf_step_clock* clock, uint64_t base_seed) {
  const int32_t t = clock->t + 1;
  clock->t = t;
  uint64_t z = base_seed + 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  clock->seed = (z ^ (z >> 31)) & 0x3FFFFFFFFFFFFFFFull;
}

__global__ void k_clock_advance(ncf_step_clock* clock, uint64_t base_seed) {
  clock_advance(clock, base_seed);
}

__global__ void k_clock_set(ncf_step_clock* clock, int32_t t, uint64_t seed) {
  clock->t = t;
  clock->reserved = 0;
  clock->seed = seed;
}

// k_adam_flat_clock + k_clock_advance in one launch: every block counts itself done in
// clock->reserved after its threads have read the clock; the last one advances the clock and
// re-arms the counter (0 between launches).
__global__ __launch_bounds__(256) void k_adam_flat_close(float* __restrict__ p,
                                                         const float* __restrict__ g,
                                                         float* __restrict__ m,
                                                         float* __restrict__ v, int64_t n,
                                                         const float* __restrict__ table,
                                                         int32_t step_rel, ncf_step_clock* clock,
                                                         uint64_t base_seed, AdamScalars s) {
  const int32_t step = clock->t + step_rel;
  const float ns = table[4 * step], bc = table[4 * step + 1];
  // float4 per lane (the flat buffers are 16-B aligned), a short scalar tail; the same adam1 per
  // element as the scalar loop (bit-identical)
  const int64_t n4 = n >> 2;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n4;
       e += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = ld4(p + 4 * e), mm = ld4(m + 4 * e), vv = ld4(v + 4 * e);
    adam4(pp, mm, vv, ld4(g + 4 * e), ns, bc, s);
    st4(p + 4 * e, pp);
    st4(m + 4 * e, mm);
    st4(v + 4 * e, vv);
  }
  if (blockIdx.x == 0 && (int64_t)threadIdx.x < n - 4 * n4) {
    const int64_t i = 4 * n4 + threadIdx.x;
    float pp = p[i], mm = m[i], vv = v[i];
    adam1(pp, mm, vv, g[i], ns, bc, s);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
  // No fence: the only ordering needed is "every block has READ the clock before it changes",
  // and a block's reads have returned before its counter increment is issued.  (A device-scope
  // release here would write the L2 back per block: measured 3x slower than two launches.)
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* done = reinterpret_cast<unsigned*>(&clock->reserved);
    if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        gridDim.x - 1) {
      *done = 0u;
      clock_advance(clock, base_seed);
    }
  }
}


int grid_for(int64_t work) {
  int64_t b = (work + 255) / 256;
  if (b > 256 * 16) b = 256 * 16;  // grid-stride beyond 16 blocks per CU
  return b < 1 ? 1 : (int)b;
}

template <int D>
int table_d(float* p, float* m, float* v, int64_t rows, const int32_t* slot, const float* G,
            const AdamScalars& s, hipStream_t st, bool bf = false) {
  if (bf)
    hipLaunchKernelGGL((k_adam_table<D, true>), dim3(grid_for(rows * (D / 4))), dim3(256), 0, st, p, m, v, rows, slot, G, s);
  else
    hipLaunchKernelGGL((k_adam_table<D, false>), dim3(grid_for(rows * (D / 4))), dim3(256), 0, st, p, m, v, rows, slot, G, s);
  NCF_CHECK_LAUNCH("ncf_adam_table");
  return NCF_OK;
}

template <int D>
int scatter_d(float* dense, const int64_t* uniq, const uint32_t* nu, int kind, const float* G,
              int64_t max_n, hipStream_t st) {
  hipLaunchKernelGGL(k_scatter_compact<D>, dim3(ncf_cdiv(max_n * (D / 4), 256)), dim3(256), 0, st,
                     dense, uniq, nu, kind, G, max_n);
  NCF_CHECK_LAUNCH("ncf_scatter_compact_rows");
  return NCF_OK;
}

}  // namespace

#define NCF_DISPATCH_DIM(D, FN, ...)                                          \
  switch (D) {                                                                \
    case 16: return FN<16>(__VA_ARGS__);                                      \
    case 32: return FN<32>(__VA_ARGS__);                                      \
    case 64: return FN<64>(__VA_ARGS__);                                      \
    case 128: return FN<128>(__VA_ARGS__);                                    \
    case 256: return FN<256>(__VA_ARGS__);                                    \
    default: ncf_set_error("unsupported dim %lld", (long long)D); return NCF_ERR_ARG; \
  }

// One Adam step over a whole [rows, dim] table (dense-exact; see header).  `slot`/`grad_compact`
// may be NULL (no touched rows: weight decay only).  `step` is the 1-based step count AFTER
// increment, as torch's state['step'].
extern "C" int ncf_adam_table(float* param, float* exp_avg, float* exp_avg_sq, int64_t rows,
                              int64_t dim, const int32_t* slot, const float* grad_compact,
                              double lr, double beta1, double beta2, double eps,
                              double weight_decay, double step, void* stream) {
  NCF_CHECK_ARG(rows >= 0 && step >= 1, "ncf_adam_table: bad args");
  if (rows == 0) return NCF_OK;
  NCF_CHECK_ARG(param && exp_avg && exp_avg_sq, "ncf_adam_table: null pointer");
  const AdamScalars s = make_scalars(lr, beta1, beta2, eps, weight_decay, step);
  NCF_DISPATCH_DIM(dim, table_d, param, exp_avg, exp_avg_sq, rows, slot, grad_compact, s,
                   (hipStream_t)stream);
}

// Adam over a flat fp32 buffer (the dense parameters, packed contiguously by the host).
extern "C" int ncf_adam_flat(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                             int64_t n, double lr, double beta1, double beta2, double eps,
                             double weight_decay, double step, void* stream) {
  NCF_CHECK_ARG(n >= 0 && step >= 1, "ncf_adam_flat: bad args");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(param && grad && exp_avg && exp_avg_sq, "ncf_adam_flat: null pointer");
  const AdamScalars s = make_scalars(lr, beta1, beta2, eps, weight_decay, step);
  hipLaunchKernelGGL(k_adam_flat, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, param,
                     grad, exp_avg, exp_avg_sq, n, s);
  NCF_CHECK_LAUNCH("ncf_adam_flat");
  return NCF_OK;
}

extern "C" int ncf_adam_table_dense_grad(float* param, const float* grad, float* exp_avg,
                                         float* exp_avg_sq, int64_t n, double lr, double beta1,
                                         double beta2, double eps, double weight_decay,
                                         double step, void* stream) {
  NCF_CHECK_ARG(n >= 0 && step >= 1, "ncf_adam_table_dense_grad: bad args");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(param && grad && exp_avg && exp_avg_sq, "ncf_adam_table_dense_grad: null pointer");
  const AdamScalars s = make_scalars(lr, beta1, beta2, eps, weight_decay, step);
  hipLaunchKernelGGL(k_adam_table_dense_grad, dim3(grid_for(n)), dim3(256), 0,
                     (hipStream_t)stream, param, grad, exp_avg, exp_avg_sq, n, s);
  NCF_CHECK_LAUNCH("ncf_adam_table_dense_grad");
  return NCF_OK;
}

extern "C" int ncf_scatter_compact_rows(float* dense_grad, int64_t dim, const int64_t* uniq,
                                        const uint32_t* num_unique, int kind,
                                        const float* grad_compact, int64_t max_n, void* stream) {
  if (max_n <= 0) return NCF_OK;
  NCF_DISPATCH_DIM(dim, scatter_d, dense_grad, uniq, num_unique, kind, grad_compact, max_n,
                   (hipStream_t)stream);
}

namespace {

template <int D>
int catchup_d(TablePtrs t, const int64_t* ids, const uint32_t* count, int kind, int64_t max_n,
              int32_t* stamp, int32_t target, const float* table, AdamScalars s,
              const ncf_step_clock* clock, hipStream_t st) {
  hipLaunchKernelGGL(k_adam_catchup<D>, dim3(ncf_cdiv(max_n * Replay<D>::LPR, 256)), dim3(256), 0, st, t,
                     ids, count, kind, max_n, stamp, target, table, s, clock);
  NCF_CHECK_LAUNCH("ncf_adam_rows_catchup");
  return NCF_OK;
}

template <int D>
int apply_d(TablePtrs t, const int64_t* ids, const uint32_t* count, int kind, int64_t max_n,
            int32_t* stamp, int32_t step, const float* table, AdamScalars s,
            const ncf_step_clock* clock, hipStream_t st) {
  hipLaunchKernelGGL(k_adam_apply<D>, dim3(ncf_cdiv(max_n * (D / 4), 256)), dim3(256), 0, st, t,
                     ids, count, kind, max_n, stamp, step, table, s, clock);
  NCF_CHECK_LAUNCH("ncf_adam_rows_apply");
  return NCF_OK;
}

template <int D>
int rolling_d(TablePtrs t, int64_t total, int64_t slice, int32_t every, int32_t* stamp,
              int32_t step_rel, const ncf_step_clock* clock, const float* table, AdamScalars s,
              hipStream_t st) {
  hipLaunchKernelGGL(k_adam_sweep_rolling<D>, dim3(grid_for(slice * Replay<D>::LPR)), dim3(256), 0, st, t,
                     total, slice, every, stamp, step_rel, clock, table, s);
  NCF_CHECK_LAUNCH("ncf_adam_sweep_rolling");
  return NCF_OK;
}

PairArgs pair_args(const ncf_table_pair* p, int n) {
  PairArgs a;
  memset(&a, 0, sizeof(a));
  for (int k = 0; k < n && k < 2; ++k) {
    a.t[k] = TablePtrs{p[k].p0, p[k].m0, p[k].v0, p[k].p1, p[k].m1, p[k].v1, p[k].g0, p[k].g1};
    a.ids[k] = p[k].row_ids;
    a.stamp[k] = p[k].stamp;
    a.rows[k] = p[k].rows;
  }
  a.bf = p[0].param_dtype == NCF_DTYPE_BF16;
  return a;
}

template <int D>
int pairs_catchup_d(PairArgs a, int n, const uint32_t* count, int64_t max_n, int32_t rel,
                    const ncf_step_clock* clock, const float* table, AdamScalars s,
                    hipStream_t st, int lock = 0) {
  if (a.bf)
    hipLaunchKernelGGL((k_pairs_catchup<D, true>), dim3(ncf_cdiv(max_n * Replay<D>::LPR, 256), n), dim3(256), 0, st, a, count, max_n, rel, clock, table, s, lock);
  else
    hipLaunchKernelGGL((k_pairs_catchup<D, false>), dim3(ncf_cdiv(max_n * Replay<D>::LPR, 256), n), dim3(256), 0, st, a, count, max_n, rel, clock, table, s, lock);
  NCF_CHECK_LAUNCH("ncf_adam_pairs_catchup_clock");
  return NCF_OK;
}

template <int D>
int pairs_apply_d(PairArgs a, int n, const uint32_t* count, int64_t max_n, int32_t rel,
                  const ncf_step_clock* clock, const float* table, AdamScalars s, hipStream_t st) {
  if (a.bf)
    hipLaunchKernelGGL((k_pairs_apply<D, true>), dim3(ncf_cdiv(max_n * (D / 4), 256), n), dim3(256), 0, st, a, count, max_n, rel, clock, table, s);
  else
    hipLaunchKernelGGL((k_pairs_apply<D, false>), dim3(ncf_cdiv(max_n * (D / 4), 256), n), dim3(256), 0, st, a, count, max_n, rel, clock, table, s);
  NCF_CHECK_LAUNCH("ncf_adam_pairs_apply_clock");
  return NCF_OK;
}

template <int D>
int pairs_apply_gsum_d(PairArgs a, int n, const uint32_t* count, int64_t max_n, int32_t rel,
                       const ncf_step_clock* clock, const float* table, AdamScalars s,
                       const float* got, const int32_t* pos0, const int32_t* pos1, int W,
                       hipStream_t st) {
  const dim3 grid(ncf_cdiv(max_n * (D / 4), 256), n);
  if (a.bf)
    hipLaunchKernelGGL((k_pairs_apply_gsum<D, true>), grid, dim3(256), 0, st, a, count, max_n, rel, clock, table, s, got, pos0, pos1, W);
  else
    hipLaunchKernelGGL((k_pairs_apply_gsum<D, false>), grid, dim3(256), 0, st, a, count, max_n, rel, clock, table, s, got, pos0, pos1, W);
  NCF_CHECK_LAUNCH("ncf_adam_pairs_apply_gsum_clock");
  return NCF_OK;
}

// blocks per CU (x 256) the rolling sweep launches at most, per kind (grid-stride beyond): the
// sweep shares the CUs with the step's kernels when it is overlapped (A/B knob,
// ncf_adam_sweep_set_blocks)
int64_t g_sweep_blocks_per_cu = 16;

template <int D>
int pairs_sweep_d(PairArgs a, int n, int32_t every, int32_t rel, const ncf_step_clock* clock,
                  const float* table, AdamScalars s, hipStream_t st, int part = 0, int nparts = 1) {
  int64_t slice = 0;
  for (int k = 0; k < n; ++k) slice = max(slice, (a.rows[k] + every - 1) / every);
  slice = (slice + nparts - 1) / nparts;
  const int gx = (int)min((int64_t)grid_for(slice * Replay<D>::LPR), 256 * g_sweep_blocks_per_cu);
  if (a.bf)
    hipLaunchKernelGGL((k_pairs_sweep<D, true>), dim3(gx, n), dim3(256), 0, st, a, every, rel, clock, table, s, part, nparts);
  else
    hipLaunchKernelGGL((k_pairs_sweep<D, false>), dim3(gx, n), dim3(256), 0, st, a, every, rel, clock, table, s, part, nparts);
  NCF_CHECK_LAUNCH("ncf_adam_pairs_sweep_rolling");
  return NCF_OK;
}

template <int D>
int sweep_d(TablePtrs t, int64_t row0, int64_t rows, int32_t* stamp, int32_t target,
            const float* table, AdamScalars s, hipStream_t st, bool bf = false) {
  if (bf)
    hipLaunchKernelGGL((k_adam_sweep<D, true>), dim3(grid_for(rows * Replay<D>::LPR)), dim3(256), 0, st, t, row0, rows, stamp, target, table, s);
  else
    hipLaunchKernelGGL((k_adam_sweep<D, false>), dim3(grid_for(rows * Replay<D>::LPR)), dim3(256), 0, st, t, row0, rows, stamp, target, table, s);
  NCF_CHECK_LAUNCH("ncf_adam_sweep");
  return NCF_OK;
}
}  // namespace

// Host helper: scalars of steps first .. first+count-1 as out[2*(s-first)] = -lr/(1-b1^s),
// out[2*(s-first)+1] = sqrt(1-b2^s) — the exact fp32 values the dense kernel uses.
extern "C" int ncf_adam_step_scalars(double lr, double beta1, double beta2, double eps,
                                     int64_t first, int64_t count, float* out_host) {
  NCF_CHECK_ARG(first >= 1 && count >= 0 && out_host, "ncf_adam_step_scalars: bad args");
  for (int64_t i = 0; i < count; ++i) {
    const AdamScalars s = make_scalars(lr, beta1, beta2, eps, 0.0, (double)(first + i));
    out_host[4 * i] = s.neg_step;
    out_host[4 * i + 1] = s.inv_bc2_sqrt;
    out_host[4 * i + 2] = s.ra;
    out_host[4 * i + 3] = s.rb;
  }
  return NCF_OK;
}

extern "C" int ncf_adam_rows_catchup(float* p0, float* m0, float* v0, float* p1, float* m1,
                                     float* v1, int64_t dim, const int64_t* row_ids,
                                     const uint32_t* count, int kind, int64_t max_n,
                                     int32_t* stamp, int32_t target, const float* step_table,
                                     double beta1, double beta2, double eps, double weight_decay,
                                     void* stream) {
  if (max_n <= 0) return NCF_OK;
  NCF_CHECK_ARG(p0 && m0 && v0 && row_ids && stamp && step_table, "ncf_adam_rows_catchup: null");
  TablePtrs t{p0, m0, v0, p1, m1, v1, nullptr, nullptr};
  NCF_DISPATCH_DIM(dim, catchup_d, t, row_ids, count, kind, max_n, stamp, target, step_table,
                   consts_of(beta1, beta2, eps, weight_decay), nullptr, (hipStream_t)stream);
}

extern "C" int ncf_adam_rows_apply(float* p0, float* m0, float* v0, const float* g0, float* p1,
                                   float* m1, float* v1, const float* g1, int64_t dim,
                                   const int64_t* row_ids, const uint32_t* count, int kind,
                                   int64_t max_n, int32_t* stamp, int32_t step,
                                   const float* step_table, double beta1, double beta2,
                                   double eps, double weight_decay, void* stream) {
  if (max_n <= 0) return NCF_OK;
  NCF_CHECK_ARG(p0 && m0 && v0 && g0 && row_ids && stamp && step_table && step >= 1,
                "ncf_adam_rows_apply: bad args");
  NCF_CHECK_ARG(!p1 || g1, "ncf_adam_rows_apply: second table without gradient");
  TablePtrs t{p0, m0, v0, p1, m1, v1, g0, g1};
  NCF_DISPATCH_DIM(dim, apply_d, t, row_ids, count, kind, max_n, stamp, step, step_table,
                   consts_of(beta1, beta2, eps, weight_decay), nullptr, (hipStream_t)stream);
}

// rows [row0, row0 + rows) caught up to `target` (a rolling sweep passes one slice per step)
extern "C" int ncf_adam_sweep(float* p0, float* m0, float* v0, float* p1, float* m1, float* v1,
                              int64_t row0, int64_t rows, int64_t dim, int32_t* stamp,
                              int32_t target, const float* step_table, double beta1, double beta2,
                              double eps, double weight_decay, void* stream) {
  if (rows <= 0) return NCF_OK;
  NCF_CHECK_ARG(p0 && m0 && v0 && stamp && step_table && row0 >= 0, "ncf_adam_sweep: bad args");
  TablePtrs t{p0, m0, v0, p1, m1, v1, nullptr, nullptr};
  NCF_DISPATCH_DIM(dim, sweep_d, t, row0, rows, stamp, target, step_table,
                   consts_of(beta1, beta2, eps, weight_decay), (hipStream_t)stream);
}

// bf16 parameter rows (fp32 moments): the same step / sweep, the parameter rounded to bf16
// (nearest even) after every step it takes
extern "C" int ncf_adam_table_bf16(uint16_t* param, float* exp_avg, float* exp_avg_sq, int64_t rows,
                                   int64_t dim, const int32_t* slot, const float* grad_compact,
                                   double lr, double beta1, double beta2, double eps,
                                   double weight_decay, double step, void* stream) {
  NCF_CHECK_ARG(rows >= 0 && step >= 1, "ncf_adam_table_bf16: bad args");
  if (rows == 0) return NCF_OK;
  NCF_CHECK_ARG(param && exp_avg && exp_avg_sq, "ncf_adam_table_bf16: null pointer");
  const AdamScalars s = make_scalars(lr, beta1, beta2, eps, weight_decay, step);
  NCF_DISPATCH_DIM(dim, table_d, reinterpret_cast<float*>(param), exp_avg, exp_avg_sq, rows, slot,
                   grad_compact, s, (hipStream_t)stream, true);
}

extern "C" int ncf_adam_sweep_bf16(uint16_t* p0, float* m0, float* v0, uint16_t* p1, float* m1,
                                   float* v1, int64_t row0, int64_t rows, int64_t dim,
                                   int32_t* stamp, int32_t target, const float* step_table,
                                   double beta1, double beta2, double eps, double weight_decay,
                                   void* stream) {
  if (rows <= 0) return NCF_OK;
  NCF_CHECK_ARG(p0 && m0 && v0 && stamp && step_table && row0 >= 0, "ncf_adam_sweep_bf16: bad args");
  TablePtrs t{reinterpret_cast<float*>(p0), m0, v0, reinterpret_cast<float*>(p1), m1, v1, nullptr,
              nullptr};
  NCF_DISPATCH_DIM(dim, sweep_d, t, row0, rows, stamp, target, step_table,
                   consts_of(beta1, beta2, eps, weight_decay), (hipStream_t)stream, true);
}

// ---- clock-driven forms (hipGraph-capturable training step)
extern "C" int ncf_step_clock_advance(ncf_step_clock* clock, uint64_t base_seed, void* stream) {
  NCF_CHECK_ARG(clock, "ncf_step_clock_advance: null clock");
  hipLaunchKernelGGL(k_clock_advance, dim3(1), dim3(1), 0, (hipStream_t)stream, clock, base_seed);
  NCF_CHECK_LAUNCH("ncf_step_clock_advance");
  return NCF_OK;
}

extern "C" int ncf_step_clock_set(ncf_step_clock* clock, int32_t t, uint64_t seed, void* stream) {
  NCF_CHECK_ARG(clock && t >= 0, "ncf_step_clock_set: null clock or t < 0");
  hipLaunchKernelGGL(k_clock_set, dim3(1), dim3(1), 0, (hipStream_t)stream, clock, t, seed);
  NCF_CHECK_LAUNCH("ncf_step_clock_set");
  return NCF_OK;
}

extern "C" int ncf_adam_rows_catchup_clock(float* p0, float* m0, float* v0, float* p1, float* m1,
                                           float* v1, int64_t dim, const int64_t* row_ids,
                                           const uint32_t* count, int kind, int64_t max_n,
                                           int32_t* stamp, int32_t target_rel,
                                           const ncf_step_clock* clock, const float* step_table,
                                           double beta1, double beta2, double eps,
                                           double weight_decay, void* stream) {
  if (max_n <= 0) return NCF_OK;
  NCF_CHECK_ARG(p0 && m0 && v0 && row_ids && stamp && step_table && clock,
                "ncf_adam_rows_catchup_clock: null");
  TablePtrs t{p0, m0, v0, p1, m1, v1, nullptr, nullptr};
  NCF_DISPATCH_DIM(dim, catchup_d, t, row_ids, count, kind, max_n, stamp, target_rel, step_table,
                   consts_of(beta1, beta2, eps, weight_decay), clock, (hipStream_t)stream);
}

extern "C" int ncf_adam_rows_apply_clock(float* p0, float* m0, float* v0, const float* g0,
                                         float* p1, float* m1, float* v1, const float* g1,
                                         int64_t dim, const int64_t* row_ids,
                                         const uint32_t* count, int kind, int64_t max_n,
                                         int32_t* stamp, int32_t step_rel,
                                         const ncf_step_clock* clock, const float* step_table,
                                         double beta1, double beta2, double eps,
                                         double weight_decay, void* stream) {
  if (max_n <= 0) return NCF_OK;
  NCF_CHECK_ARG(p0 && m0 && v0 && g0 && row_ids && stamp && step_table && clock,
                "ncf_adam_rows_apply_clock: bad args");
  NCF_CHECK_ARG(!p1 || g1, "ncf_adam_rows_apply_clock: second table without gradient");
  TablePtrs t{p0, m0, v0, p1, m1, v1, g0, g1};
  NCF_DISPATCH_DIM(dim, apply_d, t, row_ids, count, kind, max_n, stamp, step_rel, step_table,
                   consts_of(beta1, beta2, eps, weight_decay), clock, (hipStream_t)stream);
}

extern "C" int ncf_adam_sweep_rolling(float* p0, float* m0, float* v0, float* p1, float* m1,
                                      float* v1, int64_t total_rows, int64_t slice,
                                      int32_t sweep_every, int64_t dim, int32_t* stamp,
                                      int32_t step_rel, const ncf_step_clock* clock,
                                      const float* step_table, double beta1, double beta2,
                                      double eps, double weight_decay, void* stream) {
  if (total_rows <= 0 || slice <= 0) return NCF_OK;
  NCF_CHECK_ARG(p0 && m0 && v0 && stamp && step_table && clock && sweep_every >= 1,
                "ncf_adam_sweep_rolling: bad args");
  TablePtrs t{p0, m0, v0, p1, m1, v1, nullptr, nullptr};
  NCF_DISPATCH_DIM(dim, rolling_d, t, total_rows, slice, sweep_every, stamp, step_rel, clock,
                   step_table, consts_of(beta1, beta2, eps, weight_decay), (hipStream_t)stream);
}

extern "C" int ncf_adam_flat_clock(float* param, const float* grad, float* exp_avg,
                                   float* exp_avg_sq, int64_t n, const float* step_table,
                                   int32_t step_rel, const ncf_step_clock* clock, double beta1,
                                   double beta2, double eps, double weight_decay, void* stream) {
  NCF_CHECK_ARG(n >= 0, "ncf_adam_flat_clock: bad args");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && step_table && clock,
                "ncf_adam_flat_clock: null pointer");
  hipLaunchKernelGGL(k_adam_flat_clock, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     param, grad, exp_avg, exp_avg_sq, n, step_table, step_rel, clock,
                     consts_of(beta1, beta2, eps, weight_decay));
  NCF_CHECK_LAUNCH("ncf_adam_flat_clock");
  return NCF_OK;
}

extern "C" int ncf_adam_flat_clock_close(float* param, const float* grad, float* exp_avg,
                                         float* exp_avg_sq, int64_t n, const float* step_table,
                                         int32_t step_rel, ncf_step_clock* clock, double beta1,
                                         double beta2, double eps, double weight_decay,
                                         uint64_t base_seed, void* stream) {
  NCF_CHECK_ARG(n >= 1 && param && grad && exp_avg && exp_avg_sq && step_table && clock,
                "ncf_adam_flat_clock_close: bad args");
  NCF_CHECK_ARG(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
                "ncf_adam_flat_clock_close: buffers must be 16-B aligned");
  // every block's arrival is one same-address atomic on the clock word: at most 64 blocks
  // (was one per 256 elements, 328 at C2: the serialised atomics held the launch ~3 us)
  int64_t nb = ((n >> 2) + 255) / 256;
  nb = nb < 1 ? 1 : (nb > 64 ? 64 : nb);
  hipLaunchKernelGGL(k_adam_flat_close, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream,
                     param, grad, exp_avg, exp_avg_sq, n, step_table, step_rel, clock, base_seed,
                     consts_of(beta1, beta2, eps, weight_decay));
  NCF_CHECK_LAUNCH("ncf_adam_flat_clock_close");
  return NCF_OK;
}

extern "C" int ncf_adam_pairs_catchup_clock(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                            const uint32_t* count, int64_t max_n,
                                            int32_t target_rel, const ncf_step_clock* clock,
                                            const float* step_table, double beta1, double beta2,
                                            double eps, double weight_decay, void* stream) {
  NCF_CHECK_ARG(pairs && npairs >= 1 && npairs <= 2 && count && clock && step_table,
                "ncf_adam_pairs_catchup_clock: bad args");
  if (max_n <= 0) return NCF_OK;
  NCF_DISPATCH_DIM(dim, pairs_catchup_d, pair_args(pairs, npairs), npairs, count, max_n,
                   target_rel, clock, step_table, consts_of(beta1, beta2, eps, weight_decay),
                   (hipStream_t)stream);
}

// lock = 1: every listed row is also marked in flight (stamp = target | NCF_STAMP_LOCK) until the
// step's apply writes its plain stamp: a catch-up of OTHER rows running meanwhile (the next
// batch's, ahead of time on a side stream) leaves this step's rows alone.  target_rel = 1 with
// lock = 0 is that early catch-up: rows current through the step now running, whose gradient
// step is a zero-gradient one because they are not in its batch (locked rows skipped).
extern "C" int ncf_adam_pairs_catchup_lock_clock(const ncf_table_pair* pairs, int npairs,
                                                 int64_t dim, const uint32_t* count,
                                                 int64_t max_n, int32_t target_rel, int32_t lock,
                                                 const ncf_step_clock* clock,
                                                 const float* step_table, double beta1,
                                                 double beta2, double eps, double weight_decay,
                                                 void* stream) {
  NCF_CHECK_ARG(pairs && npairs >= 1 && npairs <= 2 && count && clock && step_table &&
                    (lock == 0 || lock == 1),
                "ncf_adam_pairs_catchup_lock_clock: bad args");
  if (max_n <= 0) return NCF_OK;
  NCF_DISPATCH_DIM(dim, pairs_catchup_d, pair_args(pairs, npairs), npairs, count, max_n,
                   target_rel, clock, step_table, consts_of(beta1, beta2, eps, weight_decay),
                   (hipStream_t)stream, lock);
}

template <int D>
int pairs_claim_d(PairArgs a, int npairs, const int64_t* ids0, const int64_t* ids1, int64_t n,
                  int32_t rel, const ncf_step_clock* clock, const float* table, AdamScalars s,
                  hipStream_t st) {
  const dim3 grid((unsigned)ncf_cdiv(n * Replay<D>::LPR, 256), npairs);
  if (a.bf)
    hipLaunchKernelGGL((k_pairs_catchup_claim<D, true>), grid, dim3(256), 0, st, a, ids0, ids1, n,
                       rel, clock, table, s);
  else
    hipLaunchKernelGGL((k_pairs_catchup_claim<D, false>), grid, dim3(256), 0, st, a, ids0, ids1, n,
                       rel, clock, table, s);
  NCF_CHECK_LAUNCH("ncf_adam_pairs_catchup_claim_clock");
  return NCF_OK;
}

// the catch-up of the rows of raw (not deduplicated) id lists: ids0 for pair 0, ids1 for pair 1,
// n occurrences each (k_pairs_catchup_claim)
extern "C" int ncf_adam_pairs_catchup_claim_clock(const ncf_table_pair* pairs, int npairs,
                                                  int64_t dim, const int64_t* ids0,
                                                  const int64_t* ids1, int64_t n,
                                                  int32_t target_rel, const ncf_step_clock* clock,
                                                  const float* step_table, double beta1,
                                                  double beta2, double eps, double weight_decay,
                                                  void* stream) {
  NCF_CHECK_ARG(pairs && npairs >= 1 && npairs <= 2 && ids0 && (npairs < 2 || ids1) && clock &&
                    step_table && n >= 0,
                "ncf_adam_pairs_catchup_claim_clock: bad args");
  if (n == 0) return NCF_OK;
  NCF_DISPATCH_DIM(dim, pairs_claim_d, pair_args(pairs, npairs), npairs, ids0, ids1, n,
                   target_rel, clock, step_table, consts_of(beta1, beta2, eps, weight_decay),
                   (hipStream_t)stream);
}

extern "C" int ncf_adam_pairs_apply_clock(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                          const uint32_t* count, int64_t max_n, int32_t step_rel,
                                          const ncf_step_clock* clock, const float* step_table,
                                          double beta1, double beta2, double eps,
                                          double weight_decay, void* stream) {
  NCF_CHECK_ARG(pairs && npairs >= 1 && npairs <= 2 && count && clock && step_table,
                "ncf_adam_pairs_apply_clock: bad args");
  for (int k = 0; k < npairs; ++k)
    NCF_CHECK_ARG(pairs[k].g0 && (!pairs[k].p1 || pairs[k].g1), "ncf_adam_pairs_apply_clock: gradients");
  if (max_n <= 0) return NCF_OK;
  NCF_DISPATCH_DIM(dim, pairs_apply_d, pair_args(pairs, npairs), npairs, count, max_n, step_rel,
                   clock, step_table, consts_of(beta1, beta2, eps, weight_decay),
                   (hipStream_t)stream);
}

// ncf_shard_owner_gradsum + ncf_adam_pairs_apply_clock in one launch (the pairs' g0 / g1 unused)
extern "C" int ncf_adam_pairs_apply_gsum_clock(const ncf_table_pair* pairs, int npairs,
                                               int64_t dim, const uint32_t* count, int64_t max_n,
                                               int32_t step_rel, const float* got,
                                               const int32_t* pos0, const int32_t* pos1,
                                               int world, const ncf_step_clock* clock,
                                               const float* step_table, double beta1,
                                               double beta2, double eps, double weight_decay,
                                               void* stream) {
  NCF_CHECK_ARG(pairs && npairs >= 1 && npairs <= 2 && count && clock && step_table && got &&
                    pos0 && pos1 && world >= 1,
                "ncf_adam_pairs_apply_gsum_clock: bad args");
  for (int k = 0; k < npairs; ++k)
    NCF_CHECK_ARG(pairs[k].p1, "ncf_adam_pairs_apply_gsum_clock: both tables of a pair");
  if (max_n <= 0) return NCF_OK;
  NCF_DISPATCH_DIM(dim, pairs_apply_gsum_d, pair_args(pairs, npairs), npairs, count, max_n,
                   step_rel, clock, step_table, consts_of(beta1, beta2, eps, weight_decay), got,
                   pos0, pos1, world, (hipStream_t)stream);
}

extern "C" int ncf_adam_pairs_sweep_rolling(const ncf_table_pair* pairs, int npairs, int64_t dim,
                                            int32_t sweep_every, int32_t step_rel,
                                            const ncf_step_clock* clock, const float* step_table,
                                            double beta1, double beta2, double eps,
                                            double weight_decay, void* stream) {
  NCF_CHECK_ARG(pairs && npairs >= 1 && npairs <= 2 && clock && step_table && sweep_every >= 1,
                "ncf_adam_pairs_sweep_rolling: bad args");
  NCF_DISPATCH_DIM(dim, pairs_sweep_d, pair_args(pairs, npairs), npairs, sweep_every, step_rel,
                   clock, step_table, consts_of(beta1, beta2, eps, weight_decay),
                   (hipStream_t)stream);
}

// One of `nparts` consecutive row ranges of that slice (both kinds): the parts of a step can run
// at different points of it (the overlapped sweep, deferred.py); together they are the slice.
extern "C" int ncf_adam_pairs_sweep_rolling_part(const ncf_table_pair* pairs, int npairs,
                                                 int64_t dim, int32_t sweep_every, int32_t step_rel,
                                                 int32_t part, int32_t nparts,
                                                 const ncf_step_clock* clock,
                                                 const float* step_table, double beta1,
                                                 double beta2, double eps, double weight_decay,
                                                 void* stream) {
  NCF_CHECK_ARG(pairs && npairs >= 1 && npairs <= 2 && clock && step_table && sweep_every >= 1 &&
                    nparts >= 1 && part >= 0 && part < nparts,
                "ncf_adam_pairs_sweep_rolling_part: bad args");
  NCF_DISPATCH_DIM(dim, pairs_sweep_d, pair_args(pairs, npairs), npairs, sweep_every, step_rel,
                   clock, step_table, consts_of(beta1, beta2, eps, weight_decay),
                   (hipStream_t)stream, part, nparts);
}

extern "C" int64_t ncf_adam_sweep_set_blocks(int64_t per_cu) {
  const int64_t prev = g_sweep_blocks_per_cu;
  if (per_cu > 0) g_sweep_blocks_per_cu = per_cu < 64 ? per_cu : 64;
  return prev;
}
