// Embedding backward: sparse-gradient segment-reduce for the dual (GMF + MLP) tables, fused
// with the LayerNorm backward of mf_norm / mlp_norm.
//
// Reference: the EBC lookups (src/model/architecture.py:286-287) have dense-weight backward
// (nn.EmbeddingBag sparse=False -> `_embedding_bag_dense_backward`: index sort + accumulate
// into a fresh dense [rows, D] grad every step), preceded by the LayerNorm backward of :305-306 /
// :311-312.  Here the dense [rows, D] gradient is never materialised.  On the dedup of
// dedup.hip (sorted positions, segments = unique ids, pieces = segments cut every PIECE sorted
// positions):
//   k_piece_reduce_ln  one group of L = D/4 lanes (float4 per lane) per piece (<= PIECE
//                      occurrences), 64/L pieces per wave: the group sums the upstream LN-output
//                      gradients of its piece's occurrences in position order and applies the
//                      LayerNorm backward to the sum.  LN is per-row and its backward is LINEAR in
//                      dy, and every occurrence of an id has the same input row, so
//                      sum_n LNbwd(dy_n) == sum_pieces LNbwd(sum_piece dy_n): a hot id (a Zipf
//                      head item with hundreds of occurrences) is spread over many groups instead
//                      of serialising one.  dgamma/dbeta partials per block.
//   k_piece_fixup      adds the extra pieces of multi-piece segments to the first piece's row in
//                      piece order.
// Output per kind: compact grads [num_unique, D] for the GMF and MLP tables of that kind.
// Deterministic: every sum has a fixed order.
#include "segments.h"
#include "adam_math.h"

using namespace ncf_seg;

namespace {

// The table Adam fused into the reduce (ncf_embedding_bwd_reduce_apply_clock): per kind the
// moments and stamps of the two tables (the parameters are the tables the reduce reads), the
// step clock and the per-step scalar table — the arithmetic of k_pairs_apply (adam.hip).
struct ApplyArgs {
  float* m[2][2];            // [kind][mf, mlp]
  float* v[2][2];
  float* p[2][2];            // the parameters (the reduce's table pointers, writable)
  int32_t* stamp[2];
  const ncf_step_clock* clock;
  const float* table;
  ncf_adam::AdamScalars s;
  int32_t step_rel;
  int on;
};

// Adam of row `row` of kind k with the two gradient rows (this lane's float4 of each)
template <bool BF>
__device__ __forceinline__ void apply_row(const ApplyArgs& ap, int k, int64_t row, int64_t col,
                                          int D, float4 g0, float4 g1, bool stamp_lane) {
  const int32_t step = ap.clock->t + ap.step_rel;
  const float ns = ap.table[4 * step], bc = ap.table[4 * step + 1];
  const int64_t o = row * D + col;
  float4 p0 = ldp4<BF>(ap.p[k][0], o), m0 = ld4(ap.m[k][0] + o), v0 = ld4(ap.v[k][0] + o);
  float4 p1 = ldp4<BF>(ap.p[k][1], o), m1 = ld4(ap.m[k][1] + o), v1 = ld4(ap.v[k][1] + o);
  ncf_adam::adam4(p0, m0, v0, g0, ns, bc, ap.s);
  ncf_adam::adam4(p1, m1, v1, g1, ns, bc, ap.s);
  stp4<BF>(ap.p[k][0], o, p0); st4(ap.m[k][0] + o, m0); st4(ap.v[k][0] + o, v0);
  stp4<BF>(ap.p[k][1], o, p1); st4(ap.m[k][1] + o, m1); st4(ap.v[k][1] + o, v1);
  if (stamp_lane) ap.stamp[k][row] = step;
}

// part[kind*nbr + block][0:D mf_g | D:2D mf_b | 2D:3D mlp_g | 3D:4D mlp_b]
constexpr int kPW = NCF_PIECE_WAVES;   // waves per block
// occurrence rows loaded per round (k_piece_reduce_ln; 8 measured slower: the reduce + fix-up
// 30.4-31.1 against 24.5-24.8 us in-step, the larger register set halving the resident waves)
constexpr int kRowBatch = 4;
template <int D, bool BF = false>
__global__ __launch_bounds__(64 * kPW) void k_piece_reduce_ln(
    const uint32_t* __restrict__ sv0, const uint32_t* __restrict__ sv1,
    const uint32_t* __restrict__ pstart0, const uint32_t* __restrict__ pstart1,
    const uint32_t* __restrict__ pseg0, const uint32_t* __restrict__ pseg1,
    const int64_t* __restrict__ uniq0, const int64_t* __restrict__ uniq1,
    const uint32_t* __restrict__ totals, const float* __restrict__ dy_mf0,
    const float* __restrict__ dy_mlp0, const float* __restrict__ dy_mf1,
    const float* __restrict__ dy_mlp1, const float* __restrict__ t_mf0,
    const float* __restrict__ t_mlp0, const float* __restrict__ t_mf1,
    const float* __restrict__ t_mlp1, const float* __restrict__ g_mf,
    const float* __restrict__ g_mlp, float eps, float* __restrict__ G_mf0,
    float* __restrict__ G_mlp0, float* __restrict__ G_mf1, float* __restrict__ G_mlp1,
    float* __restrict__ xp0, float* __restrict__ xp1, float* __restrict__ part,
    const int32_t* __restrict__ omap0, const int32_t* __restrict__ omap1, int64_t ldo,
    int64_t ldt, const ApplyArgs ap) {
  constexpr int L = D / 4;
  constexpr int S = 64 / L;  // lane groups (pieces) per wave
  __shared__ __attribute__((aligned(16))) float red[kPW][4 * D];
  const int32_t* omap = blockIdx.y ? omap1 : omap0;   // output row of segment c (NULL: c)
  const int kind = blockIdx.y;
  const uint32_t* sv = kind ? sv1 : sv0;
  const uint32_t* pstart = kind ? pstart1 : pstart0;
  const uint32_t* pseg = kind ? pseg1 : pseg0;
  const int64_t* uniq = kind ? uniq1 : uniq0;  // table row of each segment (caller's id space)
  const float* dmf = kind ? dy_mf1 : dy_mf0;
  const float* dml = kind ? dy_mlp1 : dy_mlp0;
  const float* tmf = kind ? t_mf1 : t_mf0;
  const float* tml = kind ? t_mlp1 : t_mlp0;
  float* Gmf = kind ? G_mf1 : G_mf0;
  float* Gml = kind ? G_mlp1 : G_mlp0;
  float* xp = kind ? xp1 : xp0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sg = lane / L, sub = lane % L;
  const int col = sub * 4;
  const int64_t Pn = totals[2 + kind];
  const float4 gm = ld4(g_mf + col), gl = ld4(g_mlp + col);
  float4 a_gm = make_float4(0, 0, 0, 0), a_bm = a_gm, a_gl = a_gm, a_bl = a_gm;
  const int64_t stride = (int64_t)gridDim.x * kPW * S;
  for (int64_t p0 = ((int64_t)blockIdx.x * kPW + w) * S; p0 < Pn; p0 += stride) {
    // the piece records (independent loads), the table rows as soon as the row is known, the
    // occurrence positions (lane sub of the group holds occurrence j0 + sub) and their rows
    const int64_t p = p0 + sg;
    const bool act = p < Pn;
    uint32_t ps = 0, info = 0;
    int cnt = 0;
    float4 x_mf = make_float4(0, 0, 0, 0), x_ml = x_mf;
    if (act) {
      ps = pstart[p];
      cnt = (int)(pstart[p + 1] - ps);  // 1..PIECE
      info = pseg[p];
      const int64_t id = uniq[info & ~FIRST_PIECE];
      x_mf = ldp4<BF>(tmf, id * ldt + col);   // (BF: bf16 table rows, widened exactly)
      x_ml = ldp4<BF>(tml, id * ldt + col);
    }
    int cmax = cnt;   // the wave's longest piece: loop bounds stay wave-uniform
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) cmax = max(cmax, __shfl_xor(cmax, o, 64));
    float4 sm = make_float4(0, 0, 0, 0), sl = sm;
    for (int j0 = 0; j0 < cmax; j0 += L) {
      const uint32_t r = (j0 + sub < cnt) ? sv[ps + j0 + sub] : 0u;
      const int jn = min(L, cmax - j0);
      // kRowBatch rows of loads in flight, summed in order
      for (int jj = 0; jj < jn; jj += kRowBatch) {
        float4 a[kRowBatch], b[kRowBatch];
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u) {
          // (jj + u < jn: a batch may run past this group's L lanes when L < kRowBatch)
          const int64_t rr = __shfl(r, sg * L + jj + u, 64);
          if (jj + u < jn && j0 + jj + u < cnt) {
            a[u] = ld4(dmf + rr * D + col);
            b[u] = ld4(dml + rr * D + col);
          }
        }
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u)
          if (jj + u < jn && j0 + jj + u < cnt) {
            sm.x += a[u].x; sm.y += a[u].y; sm.z += a[u].z; sm.w += a[u].w;
            sl.x += b[u].x; sl.y += b[u].y; sl.z += b[u].z; sl.w += b[u].w;
          }
      }
    }
    const int64_t c = info & ~FIRST_PIECE;
    const bool first = (info & FIRST_PIECE) != 0;
    // (fused apply: a segment of one piece is complete here; longer ones in the fix-up)
    const bool single = first && !(p + 1 < Pn && !(pseg[p + 1] & FIRST_PIECE));
    float4 gdx[2];
    // two LayerNorm backwards (GMF row, MLP row) per group
#pragma unroll
    for (int tbl = 0; tbl < 2; ++tbl) {
      const float4 x = tbl ? x_ml : x_mf;
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
      if (act) {
        const float4 dx = make_float4(rstd * (gd.x - m1 - h.x * m2), rstd * (gd.y - m1 - h.y * m2),
                                      rstd * (gd.z - m1 - h.z * m2), rstd * (gd.w - m1 - h.w * m2));
        float* dst = first ? (tbl ? Gml : Gmf) + (omap ? (int64_t)omap[c] : c) * ldo
                           : xp + (p - c - 1) * 2 * D + tbl * D;  // extra piece e = p - c - 1
        st4(dst + col, dx);
        gdx[tbl] = dx;
        float4& ag = tbl ? a_gl : a_gm;
        float4& ab = tbl ? a_bl : a_bm;
        ag.x += dy.x * h.x; ag.y += dy.y * h.y; ag.z += dy.z * h.z; ag.w += dy.w * h.w;
        ab.x += dy.x; ab.y += dy.y; ab.z += dy.z; ab.w += dy.w;
      }
    }
    if (ap.on && act && single)
      apply_row<BF>(ap, kind, uniq[c], col, D, gdx[0], gdx[1], sub == 0);
  }
  // the wave's groups (lanes L apart hold the same columns), then the block's waves
#pragma unroll
  for (int o = L; o < 64; o <<= 1) {
    a_gm.x += __shfl_xor(a_gm.x, o, 64); a_gm.y += __shfl_xor(a_gm.y, o, 64);
    a_gm.z += __shfl_xor(a_gm.z, o, 64); a_gm.w += __shfl_xor(a_gm.w, o, 64);
    a_bm.x += __shfl_xor(a_bm.x, o, 64); a_bm.y += __shfl_xor(a_bm.y, o, 64);
    a_bm.z += __shfl_xor(a_bm.z, o, 64); a_bm.w += __shfl_xor(a_bm.w, o, 64);
    a_gl.x += __shfl_xor(a_gl.x, o, 64); a_gl.y += __shfl_xor(a_gl.y, o, 64);
    a_gl.z += __shfl_xor(a_gl.z, o, 64); a_gl.w += __shfl_xor(a_gl.w, o, 64);
    a_bl.x += __shfl_xor(a_bl.x, o, 64); a_bl.y += __shfl_xor(a_bl.y, o, 64);
    a_bl.z += __shfl_xor(a_bl.z, o, 64); a_bl.w += __shfl_xor(a_bl.w, o, 64);
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
  for (int i = threadIdx.x; i < 4 * D; i += 64 * kPW) {
    float a = 0.0f;
#pragma unroll
    for (int q = 0; q < kPW; ++q) a += red[q][i];
    out[i] = a;
  }
}

// G[c] += extra pieces of segment c (in piece order); L lanes per segment
template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_piece_fixup(
    const uint32_t* __restrict__ fpiece0, const uint32_t* __restrict__ fpiece1,
    const uint32_t* __restrict__ totals, const float* __restrict__ xp0,
    const float* __restrict__ xp1, float* __restrict__ G_mf0, float* __restrict__ G_mlp0,
    float* __restrict__ G_mf1, float* __restrict__ G_mlp1, const int32_t* __restrict__ omap0,
    const int32_t* __restrict__ omap1, int64_t ldo, const int64_t* __restrict__ uniq0,
    const int64_t* __restrict__ uniq1, const ApplyArgs ap) {
  constexpr int L = D / 4;
  const int kind = blockIdx.y;
  const int32_t* omap = kind ? omap1 : omap0;
  const uint32_t* fpiece = kind ? fpiece1 : fpiece0;
  const float* xp = kind ? xp1 : xp0;
  float* Gmf = kind ? G_mf1 : G_mf0;
  float* Gml = kind ? G_mlp1 : G_mlp0;
  const int64_t U = totals[kind];
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int col = (int)(t % L) * 4;
  for (int64_t c = t / L; c < U; c += (int64_t)gridDim.x * blockDim.x / L) {
    const uint32_t f0 = fpiece[c], f1 = fpiece[c + 1];
    if (f1 - f0 <= 1) continue;
    const int64_t orow = (omap ? (int64_t)omap[c] : c) * ldo;
    float4 a = ld4(Gmf + orow + col), b = ld4(Gml + orow + col);
    const int64_t e1 = (int64_t)f1 - c - 1;
    for (int64_t e0 = (int64_t)f0 - c; e0 < e1; e0 += 8) {   // 8 rows of loads in flight
      float4 x[8], y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u < e1) {
          x[u] = ld4(xp + (e0 + u) * 2 * D + col);
          y[u] = ld4(xp + (e0 + u) * 2 * D + D + col);
        }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u < e1) {   // summed in piece order
          a.x += x[u].x; a.y += x[u].y; a.z += x[u].z; a.w += x[u].w;
          b.x += y[u].x; b.y += y[u].y; b.z += y[u].z; b.w += y[u].w;
        }
    }
    st4(Gmf + orow + col, a);
    st4(Gml + orow + col, b);
    if (ap.on) apply_row<BF>(ap, kind, (kind ? uniq1 : uniq0)[c], col, D, a, b, col == 0);
  }
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

template <int D>
int piece_reduce(const WS& w, int64_t n, const uint32_t* sv0, const uint32_t* sv1,
                 const int64_t* uniq0, const int64_t* uniq1, const float* dmf0, const float* dml0,
                 const float* dmf1, const float* dml1, const float* tmf0, const float* tml0,
                 const float* tmf1, const float* tml1, const float* gmf, const float* gml,
                 float eps, float* Gmf0, float* Gml0, float* Gmf1, float* Gml1, float* dgm,
                 float* dbm, float* dgl, float* dbl, ncf_reduce_list* defer, hipStream_t st,
                 bool bf = false, const int32_t* omap0 = nullptr, const int32_t* omap1 = nullptr,
                 int64_t ldo = D, int64_t ldt = D, const ApplyArgs* apply = nullptr) {
  ApplyArgs ap{};
  if (apply) ap = *apply;
  if (bf)
    hipLaunchKernelGGL((k_piece_reduce_ln<D, true>), dim3(w.nbr, 2), dim3(64 * kPW), 0, st, sv0, sv1,
                       w.pstart0, w.pstart1, w.pseg0, w.pseg1, uniq0, uniq1, w.totals,
                       dmf0, dml0, dmf1, dml1, tmf0, tml0, tmf1, tml1, gmf, gml, eps, Gmf0, Gml0,
                       Gmf1, Gml1, w.xp0, w.xp1, w.part, omap0, omap1, ldo, ldt, ap);
  else
    hipLaunchKernelGGL((k_piece_reduce_ln<D, false>), dim3(w.nbr, 2), dim3(64 * kPW), 0, st, sv0, sv1,
                       w.pstart0, w.pstart1, w.pseg0, w.pseg1, uniq0, uniq1, w.totals,
                       dmf0, dml0, dmf1, dml1, tmf0, tml0, tmf1, tml1, gmf, gml, eps, Gmf0, Gml0,
                       Gmf1, Gml1, w.xp0, w.xp1, w.part, omap0, omap1, ldo, ldt, ap);
  NCF_CHECK_LAUNCH("ncf_embedding_bwd(piece_reduce)");
  constexpr int L = D / 4;
  const int64_t fb = ncf_cdiv(n * L, 256);
  const dim3 fgrid((unsigned)(fb > 2048 ? 2048 : (fb < 1 ? 1 : fb)), 2);
  if (bf)
    hipLaunchKernelGGL((k_piece_fixup<D, true>), fgrid, dim3(256), 0, st, w.fpiece0, w.fpiece1,
                       w.totals, w.xp0, w.xp1, Gmf0, Gml0, Gmf1, Gml1, omap0, omap1, ldo, uniq0,
                       uniq1, ap);
  else
    hipLaunchKernelGGL((k_piece_fixup<D, false>), fgrid, dim3(256), 0, st, w.fpiece0, w.fpiece1,
                       w.totals, w.xp0, w.xp1, Gmf0, Gml0, Gmf1, Gml1, omap0, omap1, ldo, uniq0,
                       uniq1, ap);
  NCF_CHECK_LAUNCH("ncf_embedding_bwd(fixup)");
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

// Phase 2: per unique id, sum the LN-output gradients of its occurrences (position order) and
// apply mf_norm / mlp_norm backward; dgamma/dbeta of both norms.  Requires the workspace filled
// by ncf_dedup_ids for the same ids.
static int embedding_bwd_reduce(bool bf, int64_t n, int64_t dim, int64_t num_users,
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
                                        void* stream, const int32_t* omap0 = nullptr,
                                        const int32_t* omap1 = nullptr, int64_t ldo = 0,
                                        int64_t ldt = 0, const ApplyArgs* apply = nullptr) {
  NCF_CHECK_ARG(n >= 0 && n < (1ll << 30), "ncf_embedding_bwd_reduce: bad n");
  NCF_CHECK_ARG(dim == 16 || dim == 32 || dim == 64 || dim == 128 || dim == 256,
                "ncf_embedding_bwd_reduce: dim must be 16/32/64/128/256");
  if (workspace_bytes < ws_bytes(n, dim)) {
    ncf_set_error("ncf_embedding_bwd_reduce: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  WS w = carve(workspace, n, dim);
  uint32_t *k0, *v0, *k1, *v1;
  sorted_bufs(w, sort_passes(num_users, num_items), &k0, &v0, &k1, &v1);
  switch (dim) {
#define SEG(DD)                                                                                   \
  case DD:                                                                                        \
    return piece_reduce<DD>(w, n, v0, v1, uniq_users, uniq_items, dy_mf_user, dy_mlp_user,        \
                            dy_mf_item, dy_mlp_item, mf_user, mlp_user, mf_item, mlp_item,        \
                            mf_gamma, mlp_gamma, eps, grad_mf_user, grad_mlp_user, grad_mf_item,  \
                            grad_mlp_item, grad_mf_gamma, grad_mf_beta, grad_mlp_gamma,           \
                            grad_mlp_beta, defer, st, bf, omap0, omap1, omap0 ? ldo : DD,     \
                            ldt ? ldt : DD, apply);
    SEG(16) SEG(32) SEG(64) SEG(128) SEG(256)
#undef SEG
  }
  return NCF_ERR_ARG;
}

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
  return embedding_bwd_reduce(false, n, dim, num_users, num_items, dy_mf_user, dy_mlp_user,
                              dy_mf_item, dy_mlp_item, mf_user, mlp_user, mf_item, mlp_item,
                              mf_gamma, mlp_gamma, eps, grad_mf_user, grad_mlp_user, grad_mf_item,
                              grad_mlp_item, uniq_users, uniq_items, grad_mf_gamma, grad_mf_beta,
                              grad_mlp_gamma, grad_mlp_beta, workspace, workspace_bytes, defer,
                              stream);
}

// The same with each unique row's two gradient rows written at row out_rows[c] of row stride
// out_ld (floats) of the four output pointers (the row-sharded step: straight into its send
// buffer, [mf | mlp] halves of 2 D floats per row, instead of compact rows it then re-orders).
extern "C" int ncf_embedding_bwd_reduce_rows(
    int64_t n, int64_t dim, int64_t num_users, int64_t num_items, const float* dy_mf_user,
    const float* dy_mlp_user, const float* dy_mf_item, const float* dy_mlp_item,
    const float* mf_user, const float* mlp_user, const float* mf_item, const float* mlp_item,
    const float* mf_gamma, const float* mlp_gamma, float eps, float* grad_mf_user,
    float* grad_mlp_user, float* grad_mf_item, float* grad_mlp_item, const int64_t* uniq_users,
    const int64_t* uniq_items, const int32_t* out_rows_users, const int32_t* out_rows_items,
    int64_t out_ld, int64_t table_ld, float* grad_mf_gamma, float* grad_mf_beta,
    float* grad_mlp_gamma, float* grad_mlp_beta, void* workspace, int64_t workspace_bytes,
    ncf_reduce_list* defer, void* stream) {
  NCF_CHECK_ARG(out_rows_users && out_rows_items && out_ld >= dim && table_ld >= dim &&
                    table_ld % 4 == 0,
                "ncf_embedding_bwd_reduce_rows: out_rows, out_ld >= dim, table_ld >= dim");
  return embedding_bwd_reduce(false, n, dim, num_users, num_items, dy_mf_user, dy_mlp_user,
                              dy_mf_item, dy_mlp_item, mf_user, mlp_user, mf_item, mlp_item,
                              mf_gamma, mlp_gamma, eps, grad_mf_user, grad_mlp_user, grad_mf_item,
                              grad_mlp_item, uniq_users, uniq_items, grad_mf_gamma, grad_mf_beta,
                              grad_mlp_gamma, grad_mlp_beta, workspace, workspace_bytes, defer,
                              stream, out_rows_users, out_rows_items, out_ld, table_ld);
}

// The reduce with the deferred table Adam's apply of this step fused in (FusedTrainStep): each
// unique row's two gradient rows, once complete (in the reduce for a segment of one piece, in
// the fix-up for longer ones), step that row's parameters and moments as
// ncf_adam_pairs_apply_clock(pairs, 2, dim, num_unique, n, step_rel, ...) would, and stamp it;
// the compact gradients are still written.  pairs[k]: p0/m0/v0 (GMF), p1/m1/v1 (MLP) and stamp
// of kind k (users, items); its p0 / p1 are the tables the reduce reads (mf_*, mlp_*), its
// param_dtype says whether they are bf16.  Same bits as the reduce followed by the apply.
extern "C" int ncf_embedding_bwd_reduce_apply_clock(
    int64_t n, int64_t dim, int64_t num_users, int64_t num_items, const float* dy_mf_user,
    const float* dy_mlp_user, const float* dy_mf_item, const float* dy_mlp_item,
    const float* mf_gamma, const float* mlp_gamma, float eps, float* grad_mf_user,
    float* grad_mlp_user, float* grad_mf_item, float* grad_mlp_item, const int64_t* uniq_users,
    const int64_t* uniq_items, float* grad_mf_gamma, float* grad_mf_beta, float* grad_mlp_gamma,
    float* grad_mlp_beta, void* workspace, int64_t workspace_bytes, ncf_reduce_list* defer,
    const ncf_table_pair* pairs, int32_t step_rel, const ncf_step_clock* clock,
    const float* step_table, double beta1, double beta2, double eps_adam, double weight_decay,
    void* stream) {
  NCF_CHECK_ARG(pairs && clock && step_table, "ncf_embedding_bwd_reduce_apply_clock: bad args");
  ApplyArgs ap{};
  for (int k = 0; k < 2; ++k) {
    NCF_CHECK_ARG(pairs[k].p0 && pairs[k].m0 && pairs[k].v0 && pairs[k].p1 && pairs[k].m1 &&
                      pairs[k].v1 && pairs[k].stamp &&
                      pairs[k].param_dtype == pairs[0].param_dtype,
                  "ncf_embedding_bwd_reduce_apply_clock: incomplete table pair");
    ap.p[k][0] = pairs[k].p0; ap.m[k][0] = pairs[k].m0; ap.v[k][0] = pairs[k].v0;
    ap.p[k][1] = pairs[k].p1; ap.m[k][1] = pairs[k].m1; ap.v[k][1] = pairs[k].v1;
    ap.stamp[k] = pairs[k].stamp;
  }
  ap.clock = clock;
  ap.table = step_table;
  ap.s = ncf_adam::consts_of(beta1, beta2, eps_adam, weight_decay);
  ap.step_rel = step_rel;
  ap.on = 1;
  const bool bf = pairs[0].param_dtype == NCF_DTYPE_BF16;
  return embedding_bwd_reduce(bf, n, dim, num_users, num_items, dy_mf_user, dy_mlp_user,
                              dy_mf_item, dy_mlp_item, pairs[0].p0, pairs[0].p1, pairs[1].p0,
                              pairs[1].p1, mf_gamma, mlp_gamma, eps, grad_mf_user, grad_mlp_user,
                              grad_mf_item, grad_mlp_item, uniq_users, uniq_items, grad_mf_gamma,
                              grad_mf_beta, grad_mlp_gamma, grad_mlp_beta, workspace,
                              workspace_bytes, defer, stream, nullptr, nullptr, 0, 0, &ap);
}

// The same with bf16 table rows (the LayerNorm recompute reads them; gradients stay fp32).
extern "C" int ncf_embedding_bwd_reduce_bf16(
    int64_t n, int64_t dim, int64_t num_users, int64_t num_items, const float* dy_mf_user,
    const float* dy_mlp_user, const float* dy_mf_item, const float* dy_mlp_item,
    const uint16_t* mf_user, const uint16_t* mlp_user, const uint16_t* mf_item,
    const uint16_t* mlp_item, const float* mf_gamma, const float* mlp_gamma, float eps,
    float* grad_mf_user, float* grad_mlp_user, float* grad_mf_item, float* grad_mlp_item,
    const int64_t* uniq_users, const int64_t* uniq_items, float* grad_mf_gamma,
    float* grad_mf_beta, float* grad_mlp_gamma, float* grad_mlp_beta, void* workspace,
    int64_t workspace_bytes, ncf_reduce_list* defer, void* stream) {
  return embedding_bwd_reduce(true, n, dim, num_users, num_items, dy_mf_user, dy_mlp_user,
                              dy_mf_item, dy_mlp_item, reinterpret_cast<const float*>(mf_user),
                              reinterpret_cast<const float*>(mlp_user),
                              reinterpret_cast<const float*>(mf_item),
                              reinterpret_cast<const float*>(mlp_item), mf_gamma, mlp_gamma, eps,
                              grad_mf_user, grad_mlp_user, grad_mf_item, grad_mlp_item, uniq_users,
                              uniq_items, grad_mf_gamma, grad_mf_beta, grad_mlp_gamma,
                              grad_mlp_beta, workspace, workspace_bytes, defer, stream);
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
