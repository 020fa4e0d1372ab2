// MLP-tower row ops: ReLU -> LayerNorm -> Dropout, forward and backward.
//
// Reference: self.mlp = n x [Linear, ReLU, LayerNorm(h), Dropout(p)] (src/model/architecture.py
// :230-242, applied at :344).  The Linear (+ReLU, fused in the GEMM epilogue) is an MFMA GEMM
// (gemm.hip); this file normalises each row of width W with L = min(64, W/4) lanes per row and
// CH float4 chunks per lane (wave64: 64/L rows per wave-instruction), and in backward produces
// the pre-ReLU gradient plus deterministic per-block partial sums of dgamma/dbeta.
#include "ncf_common.h"

namespace {

template <int W>
struct Geo {
  static constexpr int L = (W / 4) < 64 ? (W / 4) : 64;  // lanes per row
  static constexpr int CH = W / (4 * L);                  // float4 chunks per lane
  static constexpr int RPW = 64 / L;                      // rows per wave-instruction
};

template <int W>
__global__ __launch_bounds__(256) void k_relu_ln_drop_fwd(float* __restrict__ r,  // [N,W] relu(lin), in
                                                          int64_t n, const float* __restrict__ g,
                                                          const float* __restrict__ b, float eps,
                                                          float p, uint64_t seed, const ncf_step_clock* clock,
                                                          float* __restrict__ out,
                                                          float* __restrict__ mean_out,
                                                          float* __restrict__ rstd_out) {
  using G = Geo<W>;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t / G::L;
  const int sub = (int)(t % G::L);
  if (row >= n) return;
  if (clock) seed += clock->seed;  // per-step stream of a captured step
  float4 x[G::CH], gg[G::CH], bb[G::CH];
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < G::CH; ++c) {
    const int col = (c * G::L + sub) * 4;
    x[c] = ld4(r + row * W + col);
    gg[c] = ld4(g + col);
    bb[c] = ld4(b + col);
    s += x[c].x + x[c].y + x[c].z + x[c].w;
  }
  const float mean = group_sum<G::L>(s) * (1.0f / W);
  float q = 0.0f;
#pragma unroll
  for (int c = 0; c < G::CH; ++c) {
    x[c].x -= mean; x[c].y -= mean; x[c].z -= mean; x[c].w -= mean;
    q += x[c].x * x[c].x + x[c].y * x[c].y + x[c].z * x[c].z + x[c].w * x[c].w;
  }
  const float rstd = 1.0f / sqrtf(group_sum<G::L>(q) * (1.0f / W) + eps);
  const float inv_keep = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
#pragma unroll
  for (int c = 0; c < G::CH; ++c) {
    const int col = (c * G::L + sub) * 4;
    float4 y = make_float4(x[c].x * rstd * gg[c].x + bb[c].x, x[c].y * rstd * gg[c].y + bb[c].y,
                           x[c].z * rstd * gg[c].z + bb[c].z, x[c].w * rstd * gg[c].w + bb[c].w);
    if (p > 0.0f) {
      const float4 k = ncf_dropout_scale4(seed, ((uint64_t)row * W + col) >> 2, p, inv_keep);
      y.x *= k.x; y.y *= k.y; y.z *= k.z; y.w *= k.w;
    }
    st4(out + row * W + col, y);
  }
  if (sub == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Backward.  Each block owns rows [blockIdx*rows_per_block, ...); partial dbias (column sums of
// the pre-ReLU gradient = bias gradient of the producing Linear) / dgamma / dbeta of the block go
// to part[blockIdx][0:W | W:2W | 2W:3W] (the order of Linear.bias, LayerNorm.weight,
// LayerNorm.bias in the parameter list, so one strided reduce lands all three).
template <int W>
__global__ __launch_bounds__(256) void k_relu_ln_drop_bwd(
    const float* __restrict__ dout, const float* __restrict__ r, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ g, int64_t n, int rows_per_block,
    float p, uint64_t seed, const ncf_step_clock* clock, float* __restrict__ dlin, float* __restrict__ part) {
  using G = Geo<W>;
  __shared__ float red[256 / G::L][3 * W];
  if (clock) seed += clock->seed;
  const int lane_grp = threadIdx.x / G::L;  // row slot inside the block iteration
  const int sub = threadIdx.x % G::L;
  const int slots = 256 / G::L;
  float4 ag[G::CH], ab[G::CH], al[G::CH];
#pragma unroll
  for (int c = 0; c < G::CH; ++c) {
    ag[c] = make_float4(0, 0, 0, 0); ab[c] = make_float4(0, 0, 0, 0); al[c] = make_float4(0, 0, 0, 0);
  }
  const float inv_keep = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  for (int64_t row = r0 + lane_grp; row < r1; row += slots) {
    const float mu = mean[row], rs = rstd[row];
    float4 dy[G::CH], xh[G::CH];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int c = 0; c < G::CH; ++c) {
      const int col = (c * G::L + sub) * 4;
      float4 d = ld4(dout + row * W + col);
      if (p > 0.0f) {
        const float4 k = ncf_dropout_scale4(seed, ((uint64_t)row * W + col) >> 2, p, inv_keep);
        d.x *= k.x; d.y *= k.y; d.z *= k.z; d.w *= k.w;
      }
      const float4 x = ld4(r + row * W + col);
      const float4 gg = ld4(g + col);
      float4 h = make_float4((x.x - mu) * rs, (x.y - mu) * rs, (x.z - mu) * rs, (x.w - mu) * rs);
      ag[c].x += d.x * h.x; ag[c].y += d.y * h.y; ag[c].z += d.z * h.z; ag[c].w += d.w * h.w;
      ab[c].x += d.x; ab[c].y += d.y; ab[c].z += d.z; ab[c].w += d.w;
      float4 gd = make_float4(d.x * gg.x, d.y * gg.y, d.z * gg.z, d.w * gg.w);
      s1 += gd.x + gd.y + gd.z + gd.w;
      s2 += gd.x * h.x + gd.y * h.y + gd.z * h.z + gd.w * h.w;
      dy[c] = gd;
      xh[c] = h;
    }
    const float m1 = group_sum<G::L>(s1) * (1.0f / W);
    const float m2 = group_sum<G::L>(s2) * (1.0f / W);
#pragma unroll
    for (int c = 0; c < G::CH; ++c) {
      const int col = (c * G::L + sub) * 4;
      const float4 x = ld4(r + row * W + col);
      float4 o;
      o.x = x.x > 0.0f ? rs * (dy[c].x - m1 - xh[c].x * m2) : 0.0f;
      o.y = x.y > 0.0f ? rs * (dy[c].y - m1 - xh[c].y * m2) : 0.0f;
      o.z = x.z > 0.0f ? rs * (dy[c].z - m1 - xh[c].z * m2) : 0.0f;
      o.w = x.w > 0.0f ? rs * (dy[c].w - m1 - xh[c].w * m2) : 0.0f;
      st4(dlin + row * W + col, o);
      al[c].x += o.x; al[c].y += o.y; al[c].z += o.z; al[c].w += o.w;
    }
  }
#pragma unroll
  for (int c = 0; c < G::CH; ++c) {
    const int col = (c * G::L + sub) * 4;
    red[lane_grp][col + 0] = al[c].x; red[lane_grp][col + 1] = al[c].y;
    red[lane_grp][col + 2] = al[c].z; red[lane_grp][col + 3] = al[c].w;
    red[lane_grp][W + col + 0] = ag[c].x; red[lane_grp][W + col + 1] = ag[c].y;
    red[lane_grp][W + col + 2] = ag[c].z; red[lane_grp][W + col + 3] = ag[c].w;
    red[lane_grp][2 * W + col + 0] = ab[c].x; red[lane_grp][2 * W + col + 1] = ab[c].y;
    red[lane_grp][2 * W + col + 2] = ab[c].z; red[lane_grp][2 * W + col + 3] = ab[c].w;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * W; i += 256) {
    float s = 0.0f;
    for (int k = 0; k < slots; ++k) s += red[k][i];
    part[(int64_t)blockIdx.x * 3 * W + i] = s;
  }
}

// rows per backward block: ~1024 blocks (enough waves in flight to hide the row loads), a
// multiple of the row slots of a block
static inline int64_t bwd_rows_per_block(int64_t n, int64_t width) {
  const int64_t L = width / 4 < 64 ? width / 4 : 64;
  const int64_t slots = 256 / L;
  int64_t rpb = (n + 1023) / 1024;
  rpb = (rpb + slots - 1) / slots * slots;
  return rpb < slots ? slots : rpb;
}

static inline int bwd_blocks(int64_t n, int64_t width) {
  return n == 0 ? 1 : (int)((n + bwd_rows_per_block(n, width) - 1) / bwd_rows_per_block(n, width));
}

template <int W>
int fwd_w(float* r, int64_t n, const float* g, const float* b, float eps, float p, uint64_t seed, const ncf_step_clock* clock,
          float* out, float* mean, float* rstd, hipStream_t st) {
  const int64_t threads = n * Geo<W>::L;
  hipLaunchKernelGGL(k_relu_ln_drop_fwd<W>, dim3(ncf_cdiv(threads, 256)), dim3(256), 0, st, r, n,
                     g, b, eps, p, seed, clock, out, mean, rstd);
  NCF_CHECK_LAUNCH("ncf_relu_ln_dropout_fwd");
  return NCF_OK;
}

template <int W>
int bwd_w(const float* dout, const float* r, const float* mean, const float* rstd, const float* g,
          int64_t n, float p, uint64_t seed, const ncf_step_clock* clock, float* dlin, float* dgamma, float* dbeta,
          float* dbias, float* ws, ncf_reduce_list* defer, hipStream_t st) {
  const int nb = bwd_blocks(n, W);
  hipLaunchKernelGGL(k_relu_ln_drop_bwd<W>, dim3(nb), dim3(256), 0, st, dout, r, mean, rstd, g, n,
                     (int)bwd_rows_per_block(n, W), p, seed, clock, dlin, ws);
  NCF_CHECK_LAUNCH("ncf_relu_ln_dropout_bwd");
  // dbias, dgamma, dbeta are the three W-wide thirds of each partial row: one strided reduce
  // when the three outputs are equally spaced (consecutive parameters of the flat buffer)
  float* scr = ws + (int64_t)nb * 3 * W;
  const ptrdiff_t s1 = dgamma - dbias, s2 = dbeta - dgamma;
  if (defer) {
    if (dbias && s1 == s2 && s1 >= W) return ncf_defer(defer, ws, nb, 3 * W, 3 * W, dbias, 0, W, s1);
    int rc = dbias ? ncf_defer(defer, ws, nb, 3 * W, W, dbias, 0, W, W) : NCF_OK;
    if (!rc) rc = ncf_defer(defer, ws + W, nb, 3 * W, W, dgamma, 0, W, W);
    if (!rc) rc = ncf_defer(defer, ws + 2 * W, nb, 3 * W, W, dbeta, 0, W, W);
    return rc;
  }
  if (dbias && s1 == s2 && s1 >= W) {
    ncf_reduce_parts(ws, nb, 3 * W, 3 * W, dbias, 0, W, s1, st, scr);
  } else {
    if (dbias) ncf_reduce_parts(ws, nb, 3 * W, W, dbias, 0, W, W, st, scr);
    ncf_reduce_parts(ws + W, nb, 3 * W, W, dgamma, 0, W, W, st, scr);
    ncf_reduce_parts(ws + 2 * W, nb, 3 * W, W, dbeta, 0, W, W, st, scr);
  }
  NCF_CHECK_LAUNCH("ncf_relu_ln_dropout_bwd(reduce)");
  return NCF_OK;
}

}  // namespace

#define NCF_DISPATCH_W(W, FN, ...)                                                   \
  switch (W) {                                                                       \
    case 16: return FN<16>(__VA_ARGS__);                                             \
    case 32: return FN<32>(__VA_ARGS__);                                             \
    case 64: return FN<64>(__VA_ARGS__);                                             \
    case 128: return FN<128>(__VA_ARGS__);                                           \
    case 256: return FN<256>(__VA_ARGS__);                                           \
    case 512: return FN<512>(__VA_ARGS__);                                           \
    case 1024: return FN<1024>(__VA_ARGS__);                                         \
    default: ncf_set_error("MLP width %lld unsupported (powers of two 16..1024)", (long long)W); \
      return NCF_ERR_ARG;                                                            \
  }

extern "C" int64_t ncf_relu_ln_dropout_bwd_workspace(int64_t n, int64_t width) {
  const int nb = bwd_blocks(n, width);
  return (int64_t)nb * 3 * width + ncf_reduce_scratch(nb, 3 * width);
}

// out = dropout(LayerNorm(r)); r already holds relu(linear) (GEMM epilogue); saves mean/rstd.
extern "C" int ncf_relu_ln_dropout_fwd(float* relu_in, int64_t n, int64_t width,
                                       const float* gamma, const float* beta, float eps,
                                       float dropout_p, uint64_t seed, const ncf_step_clock* clock, float* out, float* mean,
                                       float* rstd, void* stream) {
  NCF_CHECK_ARG(n >= 0, "ncf_relu_ln_dropout_fwd: n < 0");
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_relu_ln_dropout_fwd: bad dropout");
  if (n == 0) return NCF_OK;
  NCF_DISPATCH_W(width, fwd_w, relu_in, n, gamma, beta, eps, dropout_p, seed, clock, out, mean, rstd,
                 (hipStream_t)stream);
}

extern "C" int ncf_relu_ln_dropout_bwd(const float* grad_out, const float* relu_in,
                                       const float* mean, const float* rstd, const float* gamma,
                                       int64_t n, int64_t width, float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                                       float* grad_lin, float* grad_gamma, float* grad_beta,
                                       float* grad_bias, float* workspace,
                                       int64_t workspace_floats, ncf_reduce_list* defer,
                                       void* stream) {
  NCF_CHECK_ARG(n >= 0, "ncf_relu_ln_dropout_bwd: n < 0");
  if (workspace_floats < ncf_relu_ln_dropout_bwd_workspace(n, width)) {
    ncf_set_error("ncf_relu_ln_dropout_bwd: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  NCF_DISPATCH_W(width, bwd_w, grad_out, relu_in, mean, rstd, gamma, n, dropout_p, seed, clock, grad_lin,
                 grad_gamma, grad_beta, grad_bias, workspace, defer, (hipStream_t)stream);
}

// out[r, c] = x[r, c] * keep-scale of mask element (r, c / group) (nn.Dropout with the package's
// dropout stream: ncf_dropout_scale of index r * (cols / group) + c / group); the keep-scales
// optionally to scales[r, c / group].  group = 1: per element; group = head dim: one decision per
// (row, head) — attention-weight dropout over a single key (CategoryHierarchy's MultiHeadAttention
// on [n, D] inputs: the softmax over one key is 1, architecture.py:45-51).  In place allowed.
__global__ void k_dropout_rows(const float* x, int64_t rows, int64_t cols, int64_t group, float p,
                               uint64_t seed, float inv_keep, float* out, float* scales) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols, c = i % cols, per = cols / group;
  const int64_t m = r * per + c / group;
  const float s = ncf_dropout_scale(seed, (uint64_t)m, p, inv_keep);
  out[i] = x[i] * s;
  if (scales && c % group == 0) scales[m] = s;
}

extern "C" int ncf_dropout_rows(const float* x, int64_t rows, int64_t cols, int64_t group,
                                float dropout_p, uint64_t seed, float* out, float* scales,
                                void* stream) {
  NCF_CHECK_ARG(x && out && rows >= 0 && cols >= 1 && group >= 1 && cols % group == 0,
                "ncf_dropout_rows: bad args (cols a multiple of group)");
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_dropout_rows: dropout_p out of [0,1)");
  const int64_t n = rows * cols;
  if (n == 0) return NCF_OK;
  hipLaunchKernelGGL(k_dropout_rows, dim3((unsigned)ncf_cdiv(n, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, rows, cols, group, dropout_p, seed,
                     1.0f / (1.0f - dropout_p), out, scales);
  NCF_CHECK_LAUNCH("ncf_dropout_rows");
  return NCF_OK;
}
