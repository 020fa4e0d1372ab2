// Output head: mlp_output Linear(h_last,1), the GMF/MLP fusion Linear(2,1) + Sigmoid, and
// (optionally fused) nn.BCELoss — forward and backward.
//
// Reference: mlp_output (src/model/architecture.py:246, :345), final (:249-252, :353-354),
// mf_output (:245, :308; its inputs LN(u_mf)*LN(i_mf) come from gather_ln.hip),
// BCELoss mean with log clamp -100 (src/model/trainer.py:78, :271) and torch's BCE backward
// grad*(x-t)/max((1-x)x, 1e-12), sigmoid backward grad*(1-y)*y.
//
// One wave per row (W3 = last MLP width <= 256, D <= 256: lanes stride the columns); per-block
// partial sums of every head-parameter gradient are reduced in a fixed order (deterministic).
#include "ncf_common.h"

namespace {

constexpr int ROWS_PER_BLOCK = 16;

__global__ __launch_bounds__(256) void k_head_fwd(const float* __restrict__ a3, int64_t n, int W3,
                                                  const float* __restrict__ w_out,
                                                  const float* __restrict__ b_out,
                                                  const float* __restrict__ mf_pred,
                                                  const float* __restrict__ w_fin,
                                                  const float* __restrict__ b_fin,
                                                  float* __restrict__ mlp_pred,
                                                  float* __restrict__ prob) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= n) return;
  float s = 0.0f;
  for (int c = lane; c < W3; c += 64) s = fmaf(a3[row * W3 + c], w_out[c], s);
  s = wave_sum(s);
  if (lane == 0) {
    const float mp = s + b_out[0];
    mlp_pred[row] = mp;
    const float z = w_fin[0] * mf_pred[row] + w_fin[1] * mp + b_fin[0];
    prob[row] = 1.0f / (1.0f + expf(-z));
  }
}

// part layout per block: [W3 dw_out][D dw_mf][dwf0, dwf1, dbf, db_out, db_mf, loss]
__global__ __launch_bounds__(256) void k_head_bwd(
    const float* __restrict__ prob, const float* __restrict__ dprob,
    const float* __restrict__ targets, float inv_n, const float* __restrict__ mf_pred,
    const float* __restrict__ mlp_pred, const float* __restrict__ a3, int W3,
    const float* __restrict__ w_out, const float* __restrict__ w_fin,
    const float* __restrict__ u_mf_ln, const float* __restrict__ i_mf_ln, int D,
    const float* __restrict__ w_mf, int64_t n, float* __restrict__ da3, float* __restrict__ du_mf,
    float* __restrict__ di_mf, float* __restrict__ part) {
  __shared__ float red[4][256 + 256 + 8];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int P = W3 + D + 6;
  float aw[4] = {0, 0, 0, 0}, am[4] = {0, 0, 0, 0};
  float sw0 = 0, sw1 = 0, sbf = 0, sbo = 0, sbm = 0, sl = 0;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS_PER_BLOCK;
  const int64_t r1 = min(n, r0 + ROWS_PER_BLOCK);
  const float wf0 = w_fin[0], wf1 = w_fin[1];
  for (int64_t row = r0 + wv; row < r1; row += 4) {
    const float o = prob[row];
    float go;
    if (targets) {
      const float t = targets[row];
      go = inv_n * (o - t) / fmaxf((1.0f - o) * o, 1e-12f);
      sl += -(t * fmaxf(logf(o), -100.0f) + (1.0f - t) * fmaxf(logf(1.0f - o), -100.0f));
    } else {
      go = dprob[row];
    }
    const float dz = go * (1.0f - o) * o;
    const float dmf = dz * wf0, dml = dz * wf1;
    sw0 += dz * mf_pred[row];
    sw1 += dz * mlp_pred[row];
    sbf += dz;
    sbo += dml;
    sbm += dmf;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = lane + 64 * k;
      if (c < W3) {
        const float x = a3[row * W3 + c];
        da3[row * W3 + c] = dml * w_out[c];
        aw[k] += dml * x;
      }
      if (c < D) {
        const float u = u_mf_ln[row * D + c], it = i_mf_ln[row * D + c];
        const float gv = dmf * w_mf[c];
        du_mf[row * D + c] = gv * it;
        di_mf[row * D + c] = gv * u;
        am[k] += dmf * u * it;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = lane + 64 * k;
    if (c < W3) red[wv][c] = aw[k];
    if (c < D) red[wv][W3 + c] = am[k];
  }
  if (lane == 0) {
    red[wv][W3 + D + 0] = sw0; red[wv][W3 + D + 1] = sw1; red[wv][W3 + D + 2] = sbf;
    red[wv][W3 + D + 3] = sbo; red[wv][W3 + D + 4] = sbm; red[wv][W3 + D + 5] = sl;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += 256)
    part[(int64_t)blockIdx.x * P + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// scatter the reduced head-gradient vector red[P] into the parameter gradients
__global__ void k_head_scatter(const float* __restrict__ red, int W3, int D, float* dw_out,
                               float* db_out, float* dw_mf, float* db_mf, float* dw_fin,
                               float* db_fin, float* loss, float inv_n) {
  const int P = W3 + D + 6;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const float s = red[i];
    if (i < W3) dw_out[i] = s;
    else if (i < W3 + D) dw_mf[i - W3] = s;
    else {
      const int k = i - W3 - D;
      if (k == 0) dw_fin[0] = s;
      else if (k == 1) dw_fin[1] = s;
      else if (k == 2) db_fin[0] = s;
      else if (k == 3) db_out[0] = s;
      else if (k == 4) db_mf[0] = s;
      else if (k == 5 && loss) loss[0] = s * inv_n;
    }
  }
}

}  // namespace

extern "C" int ncf_head_fwd(const float* mlp_last, int64_t n, int64_t width, const float* mlp_out_w,
                            const float* mlp_out_b, const float* mf_pred, const float* final_w,
                            const float* final_b, float* mlp_pred, float* prob, void* stream) {
  NCF_CHECK_ARG(n >= 0 && width >= 1, "ncf_head_fwd: bad size");
  if (n == 0) return NCF_OK;
  hipLaunchKernelGGL(k_head_fwd, dim3(ncf_cdiv(n * 64, 256)), dim3(256), 0, (hipStream_t)stream,
                     mlp_last, n, (int)width, mlp_out_w, mlp_out_b, mf_pred, final_w, final_b,
                     mlp_pred, prob);
  NCF_CHECK_LAUNCH("ncf_head_fwd");
  return NCF_OK;
}

extern "C" int64_t ncf_head_bwd_workspace(int64_t n, int64_t width, int64_t dim) {
  const int nb = n == 0 ? 1 : ncf_cdiv(n, ROWS_PER_BLOCK);
  const int64_t P = width + dim + 6;
  return (int64_t)(nb + 1) * P + ncf_reduce_scratch(nb, P);
}

// Backward of the head.  Either grad_prob (upstream dL/dprob, e.g. from torch's BCELoss) or
// targets (fused mean-BCE; then *loss receives the loss value) must be given.
extern "C" int ncf_head_bwd(const float* prob, const float* grad_prob, const float* targets,
                            const float* mf_pred, const float* mlp_pred, const float* mlp_last,
                            int64_t n, int64_t width, const float* mlp_out_w, const float* final_w,
                            const float* mf_user_ln, const float* mf_item_ln, int64_t dim,
                            const float* mf_out_w, float* grad_mlp_last, float* grad_mf_user_ln,
                            float* grad_mf_item_ln, float* grad_mlp_out_w, float* grad_mlp_out_b,
                            float* grad_mf_out_w, float* grad_mf_out_b, float* grad_final_w,
                            float* grad_final_b, float* loss, double loss_denominator,
                            float* workspace, int64_t workspace_floats, ncf_reduce_list* defer,
                            void* stream) {
  NCF_CHECK_ARG(n >= 0 && width >= 1 && width <= 256 && dim >= 1 && dim <= 256,
                "ncf_head_bwd: bad size (width, dim <= 256)");
  NCF_CHECK_ARG((grad_prob != nullptr) != (targets != nullptr),
                "ncf_head_bwd: exactly one of grad_prob / targets");
  if (workspace_floats < ncf_head_bwd_workspace(n, width, dim)) {
    ncf_set_error("ncf_head_bwd: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const int nb = n == 0 ? 1 : ncf_cdiv(n, ROWS_PER_BLOCK);
  // mean over `loss_denominator` samples (the global batch under data parallelism), else over n
  const double den = loss_denominator > 0 ? loss_denominator : (double)n;
  const float inv_n = den > 0 ? (float)(1.0 / den) : 0.0f;
  hipLaunchKernelGGL(k_head_bwd, dim3(nb), dim3(256), 0, st, prob, grad_prob, targets, inv_n,
                     mf_pred, mlp_pred, mlp_last, (int)width, mlp_out_w, final_w, mf_user_ln,
                     mf_item_ln, (int)dim, mf_out_w, n, grad_mlp_last, grad_mf_user_ln,
                     grad_mf_item_ln, workspace);
  NCF_CHECK_LAUNCH("ncf_head_bwd");
  const int64_t P = width + dim + 6;
  if (defer) {  // the partial row layout of k_head_bwd, one descriptor per parameter
    const int64_t W3 = width;
    int rc = ncf_defer(defer, workspace, nb, P, W3, grad_mlp_out_w, 0, W3, W3);
    if (!rc) rc = ncf_defer(defer, workspace + W3, nb, P, dim, grad_mf_out_w, 0, dim, dim);
    if (!rc) rc = ncf_defer(defer, workspace + W3 + dim, nb, P, 2, grad_final_w, 0, 2, 2);
    if (!rc) rc = ncf_defer(defer, workspace + W3 + dim + 2, nb, P, 1, grad_final_b, 0, 1, 1);
    if (!rc) rc = ncf_defer(defer, workspace + W3 + dim + 3, nb, P, 1, grad_mlp_out_b, 0, 1, 1);
    if (!rc) rc = ncf_defer(defer, workspace + W3 + dim + 4, nb, P, 1, grad_mf_out_b, 0, 1, 1);
    if (!rc && loss) rc = ncf_defer(defer, workspace + W3 + dim + 5, nb, P, 1, loss, 0, 1, 1, inv_n);
    return rc;
  }
  float* red = workspace + (int64_t)nb * P;
  ncf_reduce_parts(workspace, nb, P, P, red, 0, P, P, st, red + P);
  hipLaunchKernelGGL(k_head_scatter, dim3(1), dim3(256), 0, st, red, (int)width, (int)dim,
                     grad_mlp_out_w, grad_mlp_out_b, grad_mf_out_w, grad_mf_out_b, grad_final_w,
                     grad_final_b, loss, inv_n);
  NCF_CHECK_LAUNCH("ncf_head_bwd(finalize)");
  return NCF_OK;
}
