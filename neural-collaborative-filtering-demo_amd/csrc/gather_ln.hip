// Embedding-row gathers fused with LayerNorm and the GMF dot product.
//
// Reference (ethanshenley/Neural-Collaborative-Filtering-Demo):
//   EBC lookups            src/model/architecture.py:286-287 (tables :153-190; single-id SUM bag == row)
//   mf_norm / mlp_norm     :305-306, :311-312 (nn.LayerNorm(D), eps 1e-5)
//   GMF                    :307-308 (mf_output Linear(D,1) of LN(u)*LN(i))
//
// Layout: tables are row-major fp32 [rows, D] (D*4-byte rows, 16-B aligned).  A row is owned by a
// group of L = D/4 lanes holding one float4 each, so a wave64 processes 64/L rows per
// instruction with fully coalesced 16-B loads; LayerNorm moments are xor-shuffle reductions
// inside the group (no LDS, no barriers).  Out-of-range ids never touch memory out of bounds:
// they read row 0 and raise bit 0 of *err (the Python layer turns that into IndexError).
#include "ncf_common.h"

// Every multiply and add below is its own IEEE operation (no fma contraction): which products the
// backend fuses depends on how the SLP vectoriser packed the float4 lanes, so the one- and
// two-float4-per-lane kernels (and ncf_gather_rows) would otherwise round differently.  With
// contraction off their arithmetic is the written expression order and their outputs are the
// same bits (tests/test_gpu_parity.py::test_gather_two_float4_lanes_bitwise_equals_one_float4).
#pragma clang fp contract(off)

namespace {

template <int D>
struct RowLN {
  static constexpr int L = D / 4;
  __device__ __forceinline__ static float4 ln(float4 x, float4 g, float4 b, float eps) {
    float s = group_sum<L>(x.x + x.y + x.z + x.w);
    float mean = s * (1.0f / D);
    float4 c = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
    float q = group_sum<L>(c.x * c.x + c.y * c.y + c.z * c.z + c.w * c.w);
    float rstd = 1.0f / sqrtf(q * (1.0f / D) + eps);
    return make_float4(c.x * rstd * g.x + b.x, c.y * rstd * g.y + b.y, c.z * rstd * g.z + b.z,
                       c.w * rstd * g.w + b.w);
  }
};

__device__ __forceinline__ int64_t safe_id(int64_t id, int64_t rows, int* err, bool report) {
  if (id < 0 || id >= rows) {
    if (err && report) atomicOr(err, 1);
    return 0;
  }
  return id;
}

template <int D, bool BF = false>
__global__ __launch_bounds__(256) void k_gather_ln_gmf(
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    const float* __restrict__ mfU, const float* __restrict__ mfI, const float* __restrict__ mlpU,
    const float* __restrict__ mlpI, int64_t nU, int64_t nI, const float* __restrict__ g_mf,
    const float* __restrict__ b_mf, const float* __restrict__ g_mlp, const float* __restrict__ b_mlp,
    const float* __restrict__ w_mf, const float* __restrict__ bias_mf, float eps,
    float* __restrict__ mf_pred, float* __restrict__ u_mlp_ln, float* __restrict__ i_mlp_ln,
    float* __restrict__ u_mf_ln, float* __restrict__ i_mf_ln, int* err,
    const float* __restrict__ item_scale, float scale_factor, int64_t G, int64_t ldt) {
  constexpr int L = D / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t / L;
  const int sub = (int)(t % L);
  if (row >= n) return;  // whole groups retire together
  const int64_t uraw = uid[row];
  const int64_t u = safe_id(uraw, nU, err, sub == 0);
  const int64_t i = safe_id(iid[row], nI, err, sub == 0);
  // G > 1 (groups of G rows, fact 6): a row whose user is its group's first row's user is that
  // row's copy — its LN'd user rows are not written (the readers take the group's first row,
  // ncf_src_row); only source rows load the user's MLP row
  const bool src = G <= 1 || row % G == 0 || uraw != uid[row - row % G];
  const int c = sub * 4;
  // (BF: the table rows are bf16; widened exactly to fp32 here, everything after is fp32)
  // (ldt: the tables' row stride in elements — D, or the row-sharded step's received rows)
  const float4 xu_mf = ldp4<BF>(mfU, u * ldt + c), xi_mf = ldp4<BF>(mfI, i * ldt + c);
  const float4 xi_ml = ldp4<BF>(mlpI, i * ldt + c);
  const float4 gm = ld4(g_mf + c), bm = ld4(b_mf + c), gl = ld4(g_mlp + c), bl = ld4(b_mlp + c);
  const float4 yu = RowLN<D>::ln(xu_mf, gm, bm, eps);
  float4 yi = RowLN<D>::ln(xi_mf, gm, bm, eps);
  float4 zi = RowLN<D>::ln(xi_ml, gl, bl, eps);
  if (item_scale) {  // forward_simple(hour): item rows *= (1 + f * proj(hour_E)) (architecture.py:444, :458)
    const float4 s4 = ld4(item_scale + row * D + c);
    const float4 m = make_float4(1.0f + scale_factor * s4.x, 1.0f + scale_factor * s4.y,
                                 1.0f + scale_factor * s4.z, 1.0f + scale_factor * s4.w);
    yi = make_float4(yi.x * m.x, yi.y * m.y, yi.z * m.z, yi.w * m.w);
    zi = make_float4(zi.x * m.x, zi.y * m.y, zi.z * m.z, zi.w * m.w);
  }
  const float4 w = ld4(w_mf + c);
  float dot = yu.x * yi.x * w.x + yu.y * yi.y * w.y + yu.z * yi.z * w.z + yu.w * yi.w * w.w;
  dot = group_sum<L>(dot);
  if (sub == 0) mf_pred[row] = dot + bias_mf[0];
  if (src) {   // (uniform in the row's lane group: its shuffles stay within active lanes)
    const float4 xu_ml = ldp4<BF>(mlpU, u * ldt + c);
    st4(u_mlp_ln + row * D + c, RowLN<D>::ln(xu_ml, gl, bl, eps));
    if (u_mf_ln) st4(u_mf_ln + row * D + c, yu);
  }
  st4(i_mlp_ln + row * D + c, zi);
  if (i_mf_ln) st4(i_mf_ln + row * D + c, yi);
}

// The same with D/8 lanes per row, each holding two float4 (columns 4k and 4k + D/2): twice the
// loads in flight per lane, half the waves, one shuffle step fewer per reduction.  Bit-identical
// to the one-float4 kernel: a lane first adds its two halves' partial sums, which is the first level of
// the D/4-lane xor tree (lane k + lane k + D/8), then the remaining levels run as before.
template <int D>
struct RowLN2 {
  static constexpr int L = D / 8;
  __device__ __forceinline__ static float s4(float4 x) { return x.x + x.y + x.z + x.w; }
  __device__ __forceinline__ static float q4(float4 c) {
    return c.x * c.x + c.y * c.y + c.z * c.z + c.w * c.w;
  }
  __device__ __forceinline__ static float4 aff(float4 c, float rstd, float4 g, float4 b) {
    return make_float4(c.x * rstd * g.x + b.x, c.y * rstd * g.y + b.y, c.z * rstd * g.z + b.z,
                       c.w * rstd * g.w + b.w);
  }
  __device__ __forceinline__ static void ln(float4& x0, float4& x1, float4 g0, float4 g1,
                                            float4 b0, float4 b1, float eps) {
    const float s = group_sum<L>(s4(x0) + s4(x1));
    const float mean = s * (1.0f / D);
    const float4 c0 = make_float4(x0.x - mean, x0.y - mean, x0.z - mean, x0.w - mean);
    const float4 c1 = make_float4(x1.x - mean, x1.y - mean, x1.z - mean, x1.w - mean);
    const float q = group_sum<L>(q4(c0) + q4(c1));
    const float rstd = 1.0f / sqrtf(q * (1.0f / D) + eps);
    x0 = aff(c0, rstd, g0, b0);
    x1 = aff(c1, rstd, g1, b1);
  }
};

// (same kernel name, third template argument = float4 per lane, so profiles keep one row for it)
template <int D, bool BF, int F4>
__global__ __launch_bounds__(256) void k_gather_ln_gmf(
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    const float* __restrict__ mfU, const float* __restrict__ mfI, const float* __restrict__ mlpU,
    const float* __restrict__ mlpI, int64_t nU, int64_t nI, const float* __restrict__ g_mf,
    const float* __restrict__ b_mf, const float* __restrict__ g_mlp, const float* __restrict__ b_mlp,
    const float* __restrict__ w_mf, const float* __restrict__ bias_mf, float eps,
    float* __restrict__ mf_pred, float* __restrict__ u_mlp_ln, float* __restrict__ i_mlp_ln,
    float* __restrict__ u_mf_ln, float* __restrict__ i_mf_ln, int* err, int64_t G, int64_t ldt) {
  static_assert(F4 == 2, "two float4 per lane");
  constexpr int L = D / 8, H2 = D / 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t / L;
  const int sub = (int)(t % L);
  if (row >= n) return;  // whole groups retire together
  const int64_t uraw = uid[row];
  const int64_t u = safe_id(uraw, nU, err, sub == 0);
  const int64_t i = safe_id(iid[row], nI, err, sub == 0);
  const bool src = G <= 1 || row % G == 0 || uraw != uid[row - row % G];
  const int c0 = sub * 4, c1 = c0 + H2;
  float4 u0 = ldp4<BF>(mfU, u * ldt + c0), u1 = ldp4<BF>(mfU, u * ldt + c1);
  float4 i0 = ldp4<BF>(mfI, i * ldt + c0), i1 = ldp4<BF>(mfI, i * ldt + c1);
  float4 z0 = ldp4<BF>(mlpI, i * ldt + c0), z1 = ldp4<BF>(mlpI, i * ldt + c1);
  float4 m0 = make_float4(0.f, 0.f, 0.f, 0.f), m1 = m0;
  if (src) {   // (uniform in the row's lane group)
    m0 = ldp4<BF>(mlpU, u * ldt + c0);
    m1 = ldp4<BF>(mlpU, u * ldt + c1);
  }
  const float4 gm0 = ld4(g_mf + c0), gm1 = ld4(g_mf + c1), bm0 = ld4(b_mf + c0), bm1 = ld4(b_mf + c1);
  const float4 gl0 = ld4(g_mlp + c0), gl1 = ld4(g_mlp + c1), bl0 = ld4(b_mlp + c0), bl1 = ld4(b_mlp + c1);
  RowLN2<D>::ln(u0, u1, gm0, gm1, bm0, bm1, eps);
  RowLN2<D>::ln(i0, i1, gm0, gm1, bm0, bm1, eps);
  RowLN2<D>::ln(z0, z1, gl0, gl1, bl0, bl1, eps);
  const float4 w0 = ld4(w_mf + c0), w1 = ld4(w_mf + c1);
  const float d0 = u0.x * i0.x * w0.x + u0.y * i0.y * w0.y + u0.z * i0.z * w0.z + u0.w * i0.w * w0.w;
  const float d1 = u1.x * i1.x * w1.x + u1.y * i1.y * w1.y + u1.z * i1.z * w1.z + u1.w * i1.w * w1.w;
  const float dot = group_sum<L>(d0 + d1);
  if (sub == 0) mf_pred[row] = dot + bias_mf[0];
  if (src) {
    RowLN2<D>::ln(m0, m1, gl0, gl1, bl0, bl1, eps);
    st4(u_mlp_ln + row * D + c0, m0);
    st4(u_mlp_ln + row * D + c1, m1);
    if (u_mf_ln) {
      st4(u_mf_ln + row * D + c0, u0);
      st4(u_mf_ln + row * D + c1, u1);
    }
  }
  st4(i_mlp_ln + row * D + c0, z0);
  st4(i_mlp_ln + row * D + c1, z1);
  if (i_mf_ln) {
    st4(i_mf_ln + row * D + c0, i0);
    st4(i_mf_ln + row * D + c1, i1);
  }
}

// Plain row gather (EBC forward as seen by callers such as app.py:156-184) with optional LN
// (get_user_embeddings / get_product_embeddings, architecture.py:383-407).
// L2 = true: each (LN'd) row divided by its Euclidean norm (the ANN export of
// generate_embeddings.py:209-211, final_vec / np.linalg.norm(final_vec))
template <int D, bool L2>
__global__ __launch_bounds__(256) void k_gather_rows_t(const int64_t* __restrict__ ids, int64_t n,
                                                     const float* __restrict__ table, int64_t rows,
                                                     const float* __restrict__ g,
                                                     const float* __restrict__ b, float eps,
                                                     float* __restrict__ out, int* err) {
  constexpr int L = D / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t / L;
  const int sub = (int)(t % L);
  if (row >= n) return;
  const int64_t id = safe_id(ids[row], rows, err, sub == 0);
  const int c = sub * 4;
  float4 x = ld4(table + id * D + c);
  if (g) x = RowLN<D>::ln(x, ld4(g + c), ld4(b + c), eps);
  if (L2) {
    const float nrm = sqrtf(group_sum<L>(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w));
    x = make_float4(x.x / nrm, x.y / nrm, x.z / nrm, x.w / nrm);
  }
  st4(out + row * D + c, x);
}

template <int D, bool BF = false>
int launch_gather_ln_gmf(const int64_t* uid, const int64_t* iid, int64_t n, const float* mfU,
                         const float* mfI, const float* mlpU, const float* mlpI, int64_t nU,
                         int64_t nI, const float* g_mf, const float* b_mf, const float* g_mlp,
                         const float* b_mlp, const float* w_mf, const float* bias_mf, float eps,
                         float* mf_pred, float* u_mlp_ln, float* i_mlp_ln, float* u_mf_ln,
                         float* i_mf_ln, int* err, const float* item_scale, float scale_factor,
                         int64_t G, hipStream_t st, int64_t ldt = D) {
  // D/8 lanes per row (the same bits; measured in-step 11.4-11.6 us either way at C2, rocprof
  // 10.1 against 10.3 us fp32 tables and 8.7 against 9.3 us bf16 tables)
  if (D >= 32 && item_scale == nullptr) {
    const int64_t threads = n * (D / 8);
    hipLaunchKernelGGL((k_gather_ln_gmf<D, BF, 2>), dim3(ncf_cdiv(threads, 256)), dim3(256), 0, st,
                       uid, iid, n, mfU, mfI, mlpU, mlpI, nU, nI, g_mf, b_mf, g_mlp, b_mlp, w_mf,
                       bias_mf, eps, mf_pred, u_mlp_ln, i_mlp_ln, u_mf_ln, i_mf_ln, err, G, ldt);
    NCF_CHECK_LAUNCH("ncf_gather_ln_gmf_fwd");
    return NCF_OK;
  }
  const int64_t threads = n * (D / 4);
  hipLaunchKernelGGL((k_gather_ln_gmf<D, BF>), dim3(ncf_cdiv(threads, 256)), dim3(256), 0, st, uid, iid,
                     n, mfU, mfI, mlpU, mlpI, nU, nI, g_mf, b_mf, g_mlp, b_mlp, w_mf, bias_mf, eps,
                     mf_pred, u_mlp_ln, i_mlp_ln, u_mf_ln, i_mf_ln, err, item_scale, scale_factor, G,
                     ldt);
  NCF_CHECK_LAUNCH("ncf_gather_ln_gmf_fwd");
  return NCF_OK;
}

template <int D>
int launch_gather_rows(const int64_t* ids, int64_t n, const float* table, int64_t rows,
                       const float* g, const float* b, float eps, float* out, int* err,
                       hipStream_t st) {
  const int64_t threads = n * (D / 4);
  hipLaunchKernelGGL((k_gather_rows_t<D, false>), dim3(ncf_cdiv(threads, 256)), dim3(256), 0, st,
                     ids, n, table, rows, g, b, eps, out, err);
  NCF_CHECK_LAUNCH("ncf_gather_rows");
  return NCF_OK;
}

template <int D>
int launch_gather_rows_l2(const int64_t* ids, int64_t n, const float* table, int64_t rows,
                          const float* g, const float* b, float eps, float* out, int* err,
                          hipStream_t st) {
  const int64_t threads = n * (D / 4);
  hipLaunchKernelGGL((k_gather_rows_t<D, true>), dim3(ncf_cdiv(threads, 256)), dim3(256), 0, st,
                     ids, n, table, rows, g, b, eps, out, err);
  NCF_CHECK_LAUNCH("ncf_embedding_export");
  return NCF_OK;
}

}  // namespace

template <int D>
int launch_gather_ln_gmf_bf16(const int64_t* uid, const int64_t* iid, int64_t n, const float* mfU,
                              const float* mfI, const float* mlpU, const float* mlpI, int64_t nU,
                              int64_t nI, const float* g_mf, const float* b_mf, const float* g_mlp,
                              const float* b_mlp, const float* w_mf, const float* bias_mf,
                              float eps, float* mf_pred, float* u_mlp_ln, float* i_mlp_ln,
                              float* u_mf_ln, float* i_mf_ln, int* err, const float* item_scale,
                              float scale_factor, int64_t G, hipStream_t st) {
  return launch_gather_ln_gmf<D, true>(uid, iid, n, mfU, mfI, mlpU, mlpI, nU, nI, g_mf, b_mf, g_mlp,
                                       b_mlp, w_mf, bias_mf, eps, mf_pred, u_mlp_ln, i_mlp_ln,
                                       u_mf_ln, i_mf_ln, err, item_scale, scale_factor, G, st);
}

#define NCF_DISPATCH_D(D, FN, ...)                                            \
  switch (D) {                                                                \
    case 16: return FN<16>(__VA_ARGS__);                                      \
    case 32: return FN<32>(__VA_ARGS__);                                      \
    case 64: return FN<64>(__VA_ARGS__);                                      \
    case 128: return FN<128>(__VA_ARGS__);                                    \
    case 256: return FN<256>(__VA_ARGS__);                                    \
    default: ncf_set_error("unsupported embedding dim %lld (16/32/64/128/256)", (long long)D); \
      return NCF_ERR_ARG;                                                     \
  }

extern "C" int ncf_gather_ln_gmf_scaled_fwd(
    const int64_t* user_ids, const int64_t* item_ids, int64_t n, const float* mf_user,
    const float* mf_item, const float* mlp_user, const float* mlp_item, int64_t num_users,
    int64_t num_items, int64_t dim, const float* mf_gamma, const float* mf_beta,
    const float* mlp_gamma, const float* mlp_beta, const float* mf_out_w, const float* mf_out_b,
    float eps, const float* item_scale, float scale_factor, int64_t group_rows, float* mf_pred,
    float* mlp_user_ln, float* mlp_item_ln, float* mf_user_ln, float* mf_item_ln, int* err_flag,
    void* stream) {
  NCF_CHECK_ARG(n >= 0 && group_rows >= 0, "ncf_gather_ln_gmf_fwd: n < 0");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(user_ids && item_ids && mf_user && mf_item && mlp_user && mlp_item && mf_pred &&
                    mlp_user_ln && mlp_item_ln && mf_gamma && mf_beta && mlp_gamma && mlp_beta &&
                    mf_out_w && mf_out_b,
                "ncf_gather_ln_gmf_fwd: null pointer");
  NCF_DISPATCH_D(dim, launch_gather_ln_gmf, user_ids, item_ids, n, mf_user, mf_item, mlp_user,
                 mlp_item, num_users, num_items, mf_gamma, mf_beta, mlp_gamma, mlp_beta, mf_out_w,
                 mf_out_b, eps, mf_pred, mlp_user_ln, mlp_item_ln, mf_user_ln, mf_item_ln,
                 err_flag, item_scale, scale_factor, group_rows, (hipStream_t)stream);
}

// The same gather over tables whose rows are table_ld elements apart (>= dim): the row-sharded
// step reads its received rows in place ([mf | mlp] halves of 2 D floats: mf_* = rows, mlp_* =
// rows + D, table_ld = 2 D) instead of copying them into compact mini tables first.
template <int D>
int launch_gather_ln_gmf_ld(const int64_t* uid, const int64_t* iid, int64_t n, const float* mfU,
                            const float* mfI, const float* mlpU, const float* mlpI, int64_t nU,
                            int64_t nI, const float* g_mf, const float* b_mf, const float* g_mlp,
                            const float* b_mlp, const float* w_mf, const float* bias_mf,
                            float eps, float* mf_pred, float* u_mlp_ln, float* i_mlp_ln,
                            float* u_mf_ln, float* i_mf_ln, int* err, int64_t G, int64_t ldt,
                            hipStream_t st) {
  return launch_gather_ln_gmf<D, false>(uid, iid, n, mfU, mfI, mlpU, mlpI, nU, nI, g_mf, b_mf,
                                        g_mlp, b_mlp, w_mf, bias_mf, eps, mf_pred, u_mlp_ln,
                                        i_mlp_ln, u_mf_ln, i_mf_ln, err, nullptr, 0.0f, G, st, ldt);
}

extern "C" int ncf_gather_ln_gmf_ld_fwd(
    const int64_t* user_ids, const int64_t* item_ids, int64_t n, const float* mf_user,
    const float* mf_item, const float* mlp_user, const float* mlp_item, int64_t num_users,
    int64_t num_items, int64_t dim, int64_t table_ld, const float* mf_gamma, const float* mf_beta,
    const float* mlp_gamma, const float* mlp_beta, const float* mf_out_w, const float* mf_out_b,
    float eps, int64_t group_rows, float* mf_pred, float* mlp_user_ln, float* mlp_item_ln,
    float* mf_user_ln, float* mf_item_ln, int* err_flag, void* stream) {
  NCF_CHECK_ARG(n >= 0 && group_rows >= 0 && table_ld >= dim && table_ld % 4 == 0,
                "ncf_gather_ln_gmf_ld_fwd: bad n / group_rows / table_ld");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(user_ids && item_ids && mf_user && mf_item && mlp_user && mlp_item && mf_pred &&
                    mlp_user_ln && mlp_item_ln && mf_gamma && mf_beta && mlp_gamma && mlp_beta &&
                    mf_out_w && mf_out_b,
                "ncf_gather_ln_gmf_ld_fwd: null pointer");
  NCF_DISPATCH_D(dim, launch_gather_ln_gmf_ld, user_ids, item_ids, n, mf_user, mf_item, mlp_user,
                 mlp_item, num_users, num_items, mf_gamma, mf_beta, mlp_gamma, mlp_beta, mf_out_w,
                 mf_out_b, eps, mf_pred, mlp_user_ln, mlp_item_ln, mf_user_ln, mf_item_ln,
                 err_flag, group_rows, table_ld, (hipStream_t)stream);
}

extern "C" int ncf_gather_ln_gmf_fwd(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                                     const float* mf_user, const float* mf_item,
                                     const float* mlp_user, const float* mlp_item,
                                     int64_t num_users, int64_t num_items, int64_t dim,
                                     const float* mf_gamma, const float* mf_beta,
                                     const float* mlp_gamma, const float* mlp_beta,
                                     const float* mf_out_w, const float* mf_out_b, float eps,
                                     float* mf_pred, float* mlp_user_ln, float* mlp_item_ln,
                                     float* mf_user_ln, float* mf_item_ln, int* err_flag,
                                     void* stream) {
  return ncf_gather_ln_gmf_scaled_fwd(user_ids, item_ids, n, mf_user, mf_item, mlp_user, mlp_item,
                                      num_users, num_items, dim, mf_gamma, mf_beta, mlp_gamma,
                                      mlp_beta, mf_out_w, mf_out_b, eps, nullptr, 0.0f, 0, mf_pred,
                                      mlp_user_ln, mlp_item_ln, mf_user_ln, mf_item_ln, err_flag,
                                      stream);
}

extern "C" int ncf_gather_rows(const int64_t* ids, int64_t n, const float* table, int64_t rows,
                               int64_t dim, const float* ln_gamma, const float* ln_beta, float eps,
                               float* out, int* err_flag, void* stream) {
  NCF_CHECK_ARG(n >= 0 && rows >= 0, "ncf_gather_rows: negative size");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(ids && table && out, "ncf_gather_rows: null pointer");
  NCF_CHECK_ARG((ln_gamma == nullptr) == (ln_beta == nullptr), "ncf_gather_rows: gamma/beta mismatch");
  NCF_DISPATCH_D(dim, launch_gather_rows, ids, n, table, rows, ln_gamma, ln_beta, eps, out,
                 err_flag, (hipStream_t)stream);
}

extern "C" int ncf_embedding_export(const int64_t* ids, int64_t n, const float* table, int64_t rows,
                                    int64_t dim, const float* ln_gamma, const float* ln_beta,
                                    float eps, int l2_normalize, float* out, int* err_flag,
                                    void* stream) {
  NCF_CHECK_ARG(n >= 0 && rows >= 0, "ncf_embedding_export: negative size");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(ids && table && out, "ncf_embedding_export: null pointer");
  NCF_CHECK_ARG((ln_gamma == nullptr) == (ln_beta == nullptr), "ncf_embedding_export: gamma/beta mismatch");
  if (!l2_normalize)
    return ncf_gather_rows(ids, n, table, rows, dim, ln_gamma, ln_beta, eps, out, err_flag, stream);
  NCF_DISPATCH_D(dim, launch_gather_rows_l2, ids, n, table, rows, ln_gamma, ln_beta, eps, out,
                 err_flag, (hipStream_t)stream);
}

// The training gather of the bf16-table configuration: the four tables hold bf16 rows (uint16
// bit patterns); LayerNorm, GMF and every output stay fp32.
extern "C" int ncf_gather_ln_gmf_bf16_fwd(
    const int64_t* user_ids, const int64_t* item_ids, int64_t n, const uint16_t* mf_user,
    const uint16_t* mf_item, const uint16_t* mlp_user, const uint16_t* mlp_item, int64_t num_users,
    int64_t num_items, int64_t dim, const float* mf_gamma, const float* mf_beta,
    const float* mlp_gamma, const float* mlp_beta, const float* mf_out_w, const float* mf_out_b,
    float eps, int64_t group_rows, float* mf_pred, float* mlp_user_ln, float* mlp_item_ln,
    float* mf_user_ln, float* mf_item_ln, int* err_flag, void* stream) {
  NCF_CHECK_ARG(n >= 0 && group_rows >= 0, "ncf_gather_ln_gmf_bf16_fwd: n < 0");
  if (n == 0) return NCF_OK;
  NCF_CHECK_ARG(user_ids && item_ids && mf_user && mf_item && mlp_user && mlp_item && mf_pred &&
                    mlp_user_ln && mlp_item_ln && mf_gamma && mf_beta && mlp_gamma && mlp_beta &&
                    mf_out_w && mf_out_b,
                "ncf_gather_ln_gmf_bf16_fwd: null pointer");
  const float* t0 = reinterpret_cast<const float*>(mf_user);
  const float* t1 = reinterpret_cast<const float*>(mf_item);
  const float* t2 = reinterpret_cast<const float*>(mlp_user);
  const float* t3 = reinterpret_cast<const float*>(mlp_item);
  NCF_DISPATCH_D(dim, launch_gather_ln_gmf_bf16, user_ids, item_ids, n, t0, t1, t2, t3, num_users,
                 num_items, mf_gamma, mf_beta, mlp_gamma, mlp_beta, mf_out_w, mf_out_b, eps,
                 mf_pred, mlp_user_ln, mlp_item_ln, mf_user_ln, mf_item_ln, err_flag, nullptr,
                 0.0f, group_rows, (hipStream_t)stream);
}
