// Host entry points of mlp_tower.hip (device code: mlp_tower_dev.h).
#include "mlp_tower_dev.h"

using namespace ncf_mlp;


#ifdef NCF_MLP_STAMPS
// diagnostic builds only (not in ncf_hip.h): copy the phase stamps [2][1024][16] to the host
extern "C" int ncf_debug_mlp_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mlp_stamps), sizeof(g_mlp_stamps)) == hipSuccess
             ? NCF_OK
             : NCF_ERR_LAUNCH;
}
#endif

extern "C" int ncf_mlp_fused_supported(int64_t dim, int64_t n_layers, const int64_t* hidden) {
  return tower_ok(dim, n_layers, hidden) ? 1 : 0;
}

template <int K0, int MM>
static void launch_fwd(const float* x, int64_t n, const TowerArgs& a, float eps, float dropout_p,
                       const ncf_step_clock* clock, const float* mlp_out_w, const float* mlp_out_b,
                       const float* mf_pred, const float* final_w, const float* final_b,
                       float* mlp_pred, float* prob, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_mlp_fwd<K0, kFwdRT, kFwdVR, MM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsFwd);
    attr = true;
  }
  hipLaunchKernelGGL((k_mlp_fwd<K0, kFwdRT, kFwdVR, MM>), dim3((unsigned)ncf_cdiv(n, kFwdVR)),
                     dim3(kThreads), kLdsFwd, st, x, n, a, eps, dropout_p, clock, mlp_out_w,
                     mlp_out_b, mf_pred, final_w, final_b, mlp_pred, prob);
}

template <int MM>
static int mlp_fwd_impl(const float* x, int64_t n, int64_t dim, const ncf_mlp_layer* layers,
                        int64_t n_layers, const int64_t* hidden, float eps, float dropout_p,
                        uint64_t seed, const ncf_step_clock* clock, const float* mlp_out_w,
                        const float* mlp_out_b, const float* mf_pred, const float* final_w,
                        const float* final_b, float* mlp_pred, float* prob, void* stream) {
  NCF_CHECK_ARG(n >= 0 && tower_ok(dim, n_layers, hidden),
                "ncf_mlp_fwd: unsupported tower (need input 64 or 128, hidden [256,128,64])");
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_mlp_fwd: dropout_p out of [0,1)");
  if (n == 0) return NCF_OK;
  TowerArgs a;
  const int rc = make_args(layers, seed, dim, a);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (dim == 64)
    launch_fwd<64, MM>(x, n, a, eps, dropout_p, clock, mlp_out_w, mlp_out_b, mf_pred, final_w,
                       final_b, mlp_pred, prob, st);
  else
    launch_fwd<128, MM>(x, n, a, eps, dropout_p, clock, mlp_out_w, mlp_out_b, mf_pred, final_w,
                        final_b, mlp_pred, prob, st);
  NCF_CHECK_LAUNCH("ncf_mlp_fwd");
  return NCF_OK;
}

// sized for the widest supported input (K0 = 128), so one workspace serves either width
extern "C" int64_t ncf_mlp_bwd_workspace(int64_t n) {
  const int64_t nb = n == 0 ? 1 : ncf_cdiv(n, kRows);
  constexpr int W = Lay<128>::kPartW;
  return nb * W + 2 * ncf_reduce_scratch((int)nb, W);
}

template <int K0, int MM>
static void launch_bwd(const float* grad_a_last, int64_t n, const TowerArgs& a, float dropout_p,
                       const ncf_step_clock* clock, float* grad_x, float* workspace,
                       const ncf_head_args& h, int fused_head, float inv_n, const float* x, int fw,
                       hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_mlp_bwd<K0, MM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
    attr = true;
  }
  hipLaunchKernelGGL((k_mlp_bwd<K0, MM>), dim3((unsigned)ncf_cdiv(n, kRows)), dim3(kThreads), kLds,
                     st, grad_a_last, n, a, dropout_p, clock, grad_x, workspace, h, fused_head,
                     inv_n, x, fw);
}

template <int MM>
static int mlp_bwd_impl(const float* grad_a_last, int64_t n, int64_t dim, const float* x,
                        const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                        float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                        const ncf_head_args* head, float* grad_x, float* workspace,
                        int64_t workspace_floats, ncf_reduce_list* defer, void* stream) {
  NCF_CHECK_ARG(n >= 0 && tower_ok(dim, n_layers, hidden),
                "ncf_mlp_bwd: unsupported tower (need input 64 or 128, hidden [256,128,64])");
  NCF_CHECK_ARG(dropout_p >= 0.0f && dropout_p < 1.0f, "ncf_mlp_bwd: dropout_p out of [0,1)");
  if (workspace_floats < ncf_mlp_bwd_workspace(n)) {
    ncf_set_error("ncf_mlp_bwd: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (n == 0) return NCF_OK;
  TowerArgs a;
  int rc = make_args(layers, seed, dim, a);
  if (rc) return rc;
  for (int l = 0; l < 3; ++l)
    if (!a.l[l].r || !a.l[l].mean || !a.l[l].rstd || !a.l[l].dgamma || !a.l[l].dbeta ||
        !a.l[l].dbias) {
      ncf_set_error("ncf_mlp_bwd: layer %d needs r/mean/rstd/dbias/dgamma/dbeta", l);
      return NCF_ERR_ARG;
    }
  const bool fw = a.l[0].dw && a.l[1].dw && a.l[2].dw;
  NCF_CHECK_ARG(fw || (a.l[0].dlin && a.l[1].dlin && a.l[2].dlin),
                "ncf_mlp_bwd: without fused weight gradients every layer needs dlin");
  NCF_CHECK_ARG(!fw || x, "ncf_mlp_bwd: fused weight gradients need x");
  ncf_head_args h{};
  float inv_n = 0.0f;
  if (head) {
    h = *head;
    NCF_CHECK_ARG((h.grad_prob != nullptr) != (h.targets != nullptr),
                  "ncf_mlp_bwd: head needs exactly one of grad_prob / targets");
    NCF_CHECK_ARG(h.prob && h.mf_pred && h.mlp_pred && h.mf_user_ln && h.mf_item_ln &&
                      h.mlp_out_w && h.final_w && h.mf_out_w && h.grad_mf_user_ln &&
                      h.grad_mf_item_ln && h.grad_mlp_out_w && h.grad_mlp_out_b &&
                      h.grad_mf_out_w && h.grad_mf_out_b && h.grad_final_w && h.grad_final_b,
                  "ncf_mlp_bwd: incomplete head arguments");
    const double den = h.loss_denominator > 0 ? h.loss_denominator : (double)n;
    inv_n = den > 0 ? (float)(1.0 / den) : 0.0f;
  } else {
    NCF_CHECK_ARG(grad_a_last != nullptr, "ncf_mlp_bwd: grad_a_last or head required");
  }
  const int nb = (int)ncf_cdiv(n, kRows);
  hipStream_t st = (hipStream_t)stream;
  if (dim == 64)
    launch_bwd<64, MM>(grad_a_last, n, a, dropout_p, clock, grad_x, workspace, h, head ? 1 : 0,
                       inv_n, x, fw ? 1 : 0, st);
  else
    launch_bwd<128, MM>(grad_a_last, n, a, dropout_p, clock, grad_x, workspace, h, head ? 1 : 0,
                        inv_n, x, fw ? 1 : 0, st);
  NCF_CHECK_LAUNCH("ncf_mlp_bwd");
  ncf_reduce_list local;
  local.count = 0;
  ncf_reduce_list* lst = defer ? defer : &local;
  rc = dim == 64 ? defer_tower<64>(a, head, h, inv_n, fw, nb, workspace, lst)
                 : defer_tower<128>(a, head, h, inv_n, fw, nb, workspace, lst);
  if (rc) return rc;
  if (!defer) {
    const int64_t PW = dim == 64 ? Lay<64>::kPartW : Lay<128>::kPartW;
    float* scr = workspace + (int64_t)nb * PW;
    return ncf_reduce_batch(lst, scr, workspace_floats - (int64_t)nb * PW, stream);
  }
  return NCF_OK;
}

extern "C" int ncf_mlp_fwd(const float* x, int64_t n, int64_t dim, const ncf_mlp_layer* layers,
                           int64_t n_layers, const int64_t* hidden, float eps, float dropout_p,
                           uint64_t seed, const ncf_step_clock* clock, const float* mlp_out_w,
                           const float* mlp_out_b, const float* mf_pred, const float* final_w,
                           const float* final_b, float* mlp_pred, float* prob, void* stream) {
  return mlp_fwd_impl<0>(x, n, dim, layers, n_layers, hidden, eps, dropout_p, seed, clock,
                             mlp_out_w, mlp_out_b, mf_pred, final_w, final_b, mlp_pred, prob,
                             stream);
}

extern "C" int ncf_mlp_bwd(const float* grad_a_last, int64_t n, int64_t dim, const float* x,
                           const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                           float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                           const ncf_head_args* head, float* grad_x, float* workspace,
                           int64_t workspace_floats, ncf_reduce_list* defer, void* stream) {
  return mlp_bwd_impl<0>(grad_a_last, n, dim, x, layers, n_layers, hidden, dropout_p, seed,
                             clock, head, grad_x, workspace, workspace_floats, defer, stream);
}

// bf16 configuration: the same tower with its three Linears (forward dX, backward dX and dW) on
// bf16 MFMA (operands rounded to bf16, fp32 accumulate); every row op stays fp32.
extern "C" int ncf_mlp_fwd_bf16(const float* x, int64_t n, int64_t dim, const ncf_mlp_layer* layers,
                                int64_t n_layers, const int64_t* hidden, float eps, float dropout_p,
                                uint64_t seed, const ncf_step_clock* clock, const float* mlp_out_w,
                                const float* mlp_out_b, const float* mf_pred, const float* final_w,
                                const float* final_b, float* mlp_pred, float* prob, void* stream) {
  return mlp_fwd_impl<1>(x, n, dim, layers, n_layers, hidden, eps, dropout_p, seed, clock,
                            mlp_out_w, mlp_out_b, mf_pred, final_w, final_b, mlp_pred, prob,
                            stream);
}

extern "C" int ncf_mlp_bwd_bf16(const float* grad_a_last, int64_t n, int64_t dim, const float* x,
                                const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                                float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                                const ncf_head_args* head, float* grad_x, float* workspace,
                                int64_t workspace_floats, ncf_reduce_list* defer, void* stream) {
  return mlp_bwd_impl<1>(grad_a_last, n, dim, x, layers, n_layers, hidden, dropout_p, seed,
                            clock, head, grad_x, workspace, workspace_floats, defer, stream);
}

// The fp32 tower with its three Linears (forward dX, backward dX and dW) on bf16 matrix cores
// through split operands (split3 / mfma_x3: six bf16 products per fp32 product, the dropped terms
// below 2^-24 of it; fp32 accumulation); every row op stays fp32.  Same arguments as ncf_mlp_fwd
// / ncf_mlp_bwd.
extern "C" int ncf_mlp_fwd_split(const float* x, int64_t n, int64_t dim, const ncf_mlp_layer* layers,
                                 int64_t n_layers, const int64_t* hidden, float eps, float dropout_p,
                                 uint64_t seed, const ncf_step_clock* clock, const float* mlp_out_w,
                                 const float* mlp_out_b, const float* mf_pred, const float* final_w,
                                 const float* final_b, float* mlp_pred, float* prob, void* stream) {
  return mlp_fwd_impl<3>(x, n, dim, layers, n_layers, hidden, eps, dropout_p, seed, clock,
                         mlp_out_w, mlp_out_b, mf_pred, final_w, final_b, mlp_pred, prob, stream);
}

extern "C" int ncf_mlp_bwd_split(const float* grad_a_last, int64_t n, int64_t dim, const float* x,
                                 const ncf_mlp_layer* layers, int64_t n_layers, const int64_t* hidden,
                                 float dropout_p, uint64_t seed, const ncf_step_clock* clock,
                                 const ncf_head_args* head, float* grad_x, float* workspace,
                                 int64_t workspace_floats, ncf_reduce_list* defer, void* stream) {
  return mlp_bwd_impl<3>(grad_a_last, n, dim, x, layers, n_layers, hidden, dropout_p, seed, clock,
                         head, grad_x, workspace, workspace_floats, defer, stream);
}
