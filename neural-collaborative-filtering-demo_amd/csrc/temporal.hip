// TemporalEncoding (src/model/architecture.py:59-94): hour/day/month embedding rows summed with
// the sinusoidal seasonal row pe[days_since mod max_period], forward and backward.
//
// Not on AdvancedNCF.forward (the reference feeds torch.zeros there, :329-334) — it is the
// op-level kernel for the temporal path (forward_simple's hour_embed, :434/:467, and the
// temporal feature views).  Forward: one L-lane group (float4 per lane) per row.  Backward into
// the three tiny tables (24/7/12 rows) is a deterministic per-(row, column) ordered reduction.
#include "ncf_common.h"

namespace {

__device__ __forceinline__ int64_t clampi(int64_t v, int64_t n, int* err) {
  if (v < 0 || v >= n) {
    if (err) atomicOr(err, 1);
    return 0;
  }
  return v;
}

__global__ void k_temporal_fwd(const int64_t* __restrict__ hour, const int64_t* __restrict__ day,
                               const int64_t* __restrict__ month, const int64_t* __restrict__ days,
                               int64_t n, const float* __restrict__ hE, const float* __restrict__ dE,
                               const float* __restrict__ mE, const float* __restrict__ pe,
                               int64_t max_period, int T, float* __restrict__ out, int* err) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t / T;
  const int c = (int)(t % T);
  if (row >= n) return;
  const int64_t h = clampi(hour[row], 24, err), d = clampi(day[row], 7, err),
                m = clampi(month[row], 12, err);
  int64_t s = days[row] % max_period;  // python-style modulo (torch %: sign of divisor)
  if (s < 0) s += max_period;
  out[row * T + c] = (hE[h * T + c] + dE[d * T + c] + mE[m * T + c]) + pe[s * T + c];
}

// grad table rows: thread per (table row r, column c), ordered loop over the batch
__global__ void k_temporal_bwd(const int64_t* __restrict__ idx, int64_t n, int rows, int T,
                               const float* __restrict__ dy, float* __restrict__ dtab) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * T) return;
  const int r = t / T, c = t % T;
  float s = 0.0f;
  for (int64_t i = 0; i < n; ++i)
    if (idx[i] == r) s += dy[i * T + c];
  dtab[t] = s;
}

}  // namespace

extern "C" int ncf_temporal_fwd(const int64_t* hour, const int64_t* day, const int64_t* month,
                                const int64_t* days_since, int64_t n, const float* hour_embed,
                                const float* day_embed, const float* month_embed, const float* pe,
                                int64_t max_period, int64_t dim, float* out, int* err_flag,
                                void* stream) {
  NCF_CHECK_ARG(n >= 0 && dim >= 1 && max_period >= 1, "ncf_temporal_fwd: bad size");
  if (n == 0) return NCF_OK;
  hipLaunchKernelGGL(k_temporal_fwd, dim3(ncf_cdiv(n * dim, 256)), dim3(256), 0,
                     (hipStream_t)stream, hour, day, month, days_since, n, hour_embed, day_embed,
                     month_embed, pe, max_period, (int)dim, out, err_flag);
  NCF_CHECK_LAUNCH("ncf_temporal_fwd");
  return NCF_OK;
}

extern "C" int ncf_temporal_bwd(const int64_t* hour, const int64_t* day, const int64_t* month,
                                int64_t n, const float* grad_out, int64_t dim, float* grad_hour,
                                float* grad_day, float* grad_month, void* stream) {
  NCF_CHECK_ARG(n >= 0 && dim >= 1, "ncf_temporal_bwd: bad size");
  hipStream_t st = (hipStream_t)stream;
  const int T = (int)dim;
  hipLaunchKernelGGL(k_temporal_bwd, dim3(ncf_cdiv(24 * T, 256)), dim3(256), 0, st, hour, n, 24, T,
                     grad_out, grad_hour);
  hipLaunchKernelGGL(k_temporal_bwd, dim3(ncf_cdiv(7 * T, 256)), dim3(256), 0, st, day, n, 7, T,
                     grad_out, grad_day);
  hipLaunchKernelGGL(k_temporal_bwd, dim3(ncf_cdiv(12 * T, 256)), dim3(256), 0, st, month, n, 12,
                     T, grad_out, grad_month);
  NCF_CHECK_LAUNCH("ncf_temporal_bwd");
  return NCF_OK;
}
