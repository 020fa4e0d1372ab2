// Ranking / classification metrics over [B, M] groups on the GPU.
//
// Reference: src/utils/metrics.py — calculate_metrics (:9-110) reshapes predictions/targets to
// [batch_size, M] and loops over users in Python: hit_rate@k (:112-137, any target == 1 among
// the top k), ndcg@k (:139-177, DCG of the relevances at ranks 1..k over log2(rank + 1), divided
// by the ideal DCG of the row's targets sorted descending; 0 when that is <= 0), mrr@k (:179-204,
// 1 / rank of the first target == 1 within the top k), map@k (:206-241, mean over the relevant
// top-k ranks of precision@rank), k clamped to M; accuracy (:258-266, (pred >= 0.5) == target)
// and its positive / negative subsets; AUC via sklearn's roc_auc_score (:243-256).
//
// ncf_group_metrics: one lane per group row; the row's rank order is (prediction desc, column
// asc) — the reference's torch.topk / torch.sort leave tie order unspecified.  Per-block double
// partial sums, then one ordered reduction (deterministic).
// ncf_auc_count: the Mann-Whitney form of roc_auc_score (ties count one half): with the negative
// predictions sorted ascending, each positive adds lo + hi = #neg < s + #neg <= s (two binary
// searches); the integer sum 2U lands in one uint64 (atomics on integers: order-independent).
#include "ncf_common.h"

namespace {

constexpr int kMaxGroup = 64;
constexpr int kMaxK = 16;

__global__ __launch_bounds__(256) void k_group_metrics(const float* __restrict__ pred,
                                                       const float* __restrict__ targ, int64_t B,
                                                       int M, const int32_t* __restrict__ ks,
                                                       int nk, float thr,
                                                       double* __restrict__ part) {
  // part[block][f]: f = 4*j + {0 hit, 1 ndcg, 2 mrr, 3 map} for k = ks[j]; then
  // 4nk + {0 correct, 1 n_pos, 2 correct_pos, 3 n_neg, 4 correct_neg}
  const int nf = 4 * nk + 5;
  __shared__ double red[256 / 64][4 * kMaxK + 5];
  double acc[4 * kMaxK + 5];
  for (int f = 0; f < nf; ++f) acc[f] = 0.0;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    const float* p = pred + b * M;
    const float* t = targ + b * M;
    float rel[kMaxGroup], ideal[kMaxGroup];
    // rank of column j: # columns ahead of it in (prediction desc, column asc)
    for (int j = 0; j < M; ++j) {
      const float pj = p[j];
      int r = 0;
      for (int i = 0; i < M; ++i) {
        const float pi = p[i];
        r += (pi > pj || (pi == pj && i < j)) ? 1 : 0;
      }
      rel[r] = t[j];
      ideal[j] = t[j];
      const bool pos = t[j] == 1.0f, neg = t[j] == 0.0f;
      const bool ok = (pj >= thr) == (t[j] != 0.0f) && (t[j] == 0.0f || t[j] == 1.0f);
      acc[4 * nk + 0] += ok ? 1.0 : 0.0;
      acc[4 * nk + 1] += pos ? 1.0 : 0.0;
      acc[4 * nk + 2] += (pos && ok) ? 1.0 : 0.0;
      acc[4 * nk + 3] += neg ? 1.0 : 0.0;
      acc[4 * nk + 4] += (neg && ok) ? 1.0 : 0.0;
    }
    // ideal order: targets descending (insertion sort, M <= 64)
    for (int i = 1; i < M; ++i) {
      const float v = ideal[i];
      int j = i - 1;
      while (j >= 0 && ideal[j] < v) { ideal[j + 1] = ideal[j]; --j; }
      ideal[j + 1] = v;
    }
    for (int q = 0; q < nk; ++q) {
      const int k = ks[q] < M ? ks[q] : M;
      double hit = 0.0, dcg = 0.0, idcg = 0.0, rr = 0.0, ap = 0.0, cnt = 0.0, cum = 0.0;
      for (int r = 0; r < k; ++r) {
        const double disc = 1.0 / log2((double)r + 2.0);
        dcg += (double)rel[r] * disc;
        idcg += (double)ideal[r] * disc;
        if (rel[r] == 1.0f) {
          if (hit == 0.0) rr = 1.0 / (r + 1.0);
          hit = 1.0;
          cum += 1.0;
          ap += cum / (r + 1.0);
          cnt += 1.0;
        }
      }
      acc[4 * q + 0] += hit;
      acc[4 * q + 1] += idcg <= 0.0 ? 0.0 : dcg / idcg;
      acc[4 * q + 2] += rr;
      acc[4 * q + 3] += cnt > 0.0 ? ap / cnt : 0.0;
    }
  }
  // block sum: waves reduce by shuffles, then wave 0 adds the 4 wave sums in order
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int f = 0; f < nf; ++f) {
    double v = acc[f];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][f] = v;
  }
  __syncthreads();
  if (threadIdx.x < nf) {
    double s = 0.0;
    for (int w = 0; w < 4; ++w) s += red[w][threadIdx.x];
    part[(int64_t)blockIdx.x * nf + threadIdx.x] = s;
  }
}

__global__ void k_sum_partials_f64(const double* __restrict__ part, int parts, int nf,
                                   double* __restrict__ out) {
  const int f = threadIdx.x;
  if (f >= nf) return;
  double s = 0.0;
  for (int p = 0; p < parts; ++p) s += part[(int64_t)p * nf + f];
  out[f] = s;
}

__global__ __launch_bounds__(256) void k_auc_count(const float* __restrict__ pred,
                                                   const float* __restrict__ targ, int64_t n,
                                                   const float* __restrict__ neg_sorted,
                                                   int64_t n_neg,
                                                   unsigned long long* __restrict__ sum2u) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long v = 0ull;
  if (i < n && targ[i] == 1.0f) {
    const float s = pred[i];
    int64_t lo = 0, hi = n_neg;   // first index with neg >= s
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (neg_sorted[m] < s) lo = m + 1;
      else hi = m;
    }
    int64_t lo2 = lo, hi2 = n_neg;   // first index with neg > s
    while (lo2 < hi2) {
      const int64_t m = (lo2 + hi2) >> 1;
      if (neg_sorted[m] <= s) lo2 = m + 1;
      else hi2 = m;
    }
    v = (unsigned long long)(lo + lo2);
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(sum2u, v);
}

}  // namespace

extern "C" int64_t ncf_group_metrics_workspace(int64_t groups, int64_t nk) {
  const int64_t nb = groups <= 0 ? 1 : ncf_cdiv(groups, 256);
  return (int64_t)sizeof(double) * nb * (4 * nk + 5);
}

extern "C" int ncf_group_metrics(const float* pred, const float* targets, int64_t groups,
                                 int64_t group_len, const int32_t* ks, int64_t nk, float threshold,
                                 double* out, void* workspace, int64_t workspace_bytes,
                                 void* stream) {
  NCF_CHECK_ARG(groups >= 0 && group_len >= 1 && group_len <= kMaxGroup,
                "ncf_group_metrics: group length must be in [1, %d]", kMaxGroup);
  NCF_CHECK_ARG(nk >= 1 && nk <= kMaxK, "ncf_group_metrics: 1..%d k values", kMaxK);
  NCF_CHECK_ARG(workspace_bytes >= ncf_group_metrics_workspace(groups, nk),
                "ncf_group_metrics: workspace too small");
  const int nf = (int)(4 * nk + 5);
  hipStream_t st = (hipStream_t)stream;
  if (groups == 0) {
    (void)hipMemsetAsync(out, 0, sizeof(double) * nf, st);
    return NCF_OK;
  }
  const int nb = (int)ncf_cdiv(groups, 256);
  double* part = (double*)workspace;
  hipLaunchKernelGGL(k_group_metrics, dim3(nb), dim3(256), 0, st, pred, targets, groups,
                     (int)group_len, ks, (int)nk, threshold, part);
  hipLaunchKernelGGL(k_sum_partials_f64, dim3(1), dim3(128), 0, st, part, nb, nf, out);
  NCF_CHECK_LAUNCH("ncf_group_metrics");
  return NCF_OK;
}

extern "C" int ncf_auc_count(const float* pred, const float* targets, int64_t n,
                             const float* neg_sorted, int64_t n_neg,
                             unsigned long long* sum_2u, void* stream) {
  NCF_CHECK_ARG(n >= 0 && n_neg >= 0, "ncf_auc_count: negative size");
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(sum_2u, 0, sizeof(unsigned long long), st);
  if (n == 0) return NCF_OK;
  hipLaunchKernelGGL(k_auc_count, dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, pred, targets, n,
                     neg_sorted, n_neg, sum_2u);
  NCF_CHECK_LAUNCH("ncf_auc_count");
  return NCF_OK;
}
