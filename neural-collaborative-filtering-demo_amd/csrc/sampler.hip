// Device-side training-batch builder: inverse-popularity negative sampling with rejection of the
// user's positives, and the single-id-bag KJT rows the model consumes.
//
// Reference: SheetzDataset (src/model/data_prep.py): product weights = 1 / max(count, 1),
// normalised (:95-102); _sample_negative (:134-161) draws np.random.choice(p=weights) up to 10
// times, rejecting the positive product and the user's history, then falls back to a uniform
// pick among the products outside the history (or, when the user has bought everything, any
// product but the positive); __getitem__ (:181-228) emits [user]*(1+k), [pos] + negatives,
// targets [1, 0, ..., 0]; collate_recommender_batch (:230-313) concatenates the batch into
// KJT values [users || items] with lengths 1.
//
// Here: the weights become a Walker/Vose alias table (built once on the host, ncf_alias_build),
// so a draw is O(1): column c = floor(u1 * I), item = u2 < prob[c] ? c : alias[c].  The history
// is a CSR of sorted item ids per user (membership by binary search).  One lane per negative;
// uniforms from the counter hash of (seed, negative index, attempt), so a batch is a pure
// function of (interaction indices, seed).  The numpy draw order of the reference is not
// reproducible (excluded from parity); the distribution and the rejection rule are.
#include "ncf_common.h"

#include <vector>

namespace {

__device__ __forceinline__ float u01(uint64_t h, int field) {   // 24-bit uniform in [0, 1)
  return (float)((uint32_t)(h >> (32 * field)) >> 8) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ bool in_sorted(const int32_t* __restrict__ a, int64_t lo, int64_t hi,
                                          int32_t x) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int32_t v = a[mid];
    if (v == x) return true;
    if (v < x) lo = mid + 1;
    else hi = mid;
  }
  return false;
}

__global__ void k_negatives(const int64_t* __restrict__ users, const int64_t* __restrict__ pos,
                            int64_t B, int k, const float* __restrict__ aprob,
                            const int32_t* __restrict__ alias, int64_t I,
                            const int64_t* __restrict__ hoff, const int32_t* __restrict__ hitem,
                            int64_t U, uint64_t seed, int max_attempts,
                            int64_t* __restrict__ out_u, int64_t* __restrict__ out_i,
                            float* __restrict__ out_t, int* __restrict__ err) {
  const int M = k + 1;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * M) return;
  const int64_t b = t / M;
  const int j = (int)(t % M);
  int64_t u = users[b];
  const int64_t p = pos[b];
  if (u < 0 || u >= U || p < 0 || p >= I) {
    atomicOr(err, 1);
    u = 0;
  }
  out_u[t] = u;
  out_t[t] = j == 0 ? 1.0f : 0.0f;
  if (j == 0) {
    out_i[t] = p;
    return;
  }
  const int64_t h0 = hoff ? hoff[u] : 0, h1 = hoff ? hoff[u + 1] : 0;
  const uint64_t neg = (uint64_t)b * (uint64_t)k + (uint64_t)(j - 1);
  for (int a = 0; a < max_attempts; ++a) {
    const uint64_t h = ncf_hash64(seed, neg * 64u + (uint64_t)a);
    int64_t c = (int64_t)(u01(h, 0) * (float)I);
    if (c >= I) c = I - 1;
    const int64_t item = u01(h, 1) < aprob[c] ? c : (int64_t)alias[c];
    if (item != p && !in_sorted(hitem, h0, h1, (int32_t)item)) {
      out_i[t] = item;
      return;
    }
  }
  // fallback (data_prep.py:153-161): uniform over the products outside history + {positive}
  const uint64_t h = ncf_hash64(seed ^ 0x5DEECE66Dull, neg);
  const int64_t nh = h1 - h0;
  const bool p_in = in_sorted(hitem, h0, h1, (int32_t)p);
  const int64_t valid = I - nh - (p_in ? 0 : 1);
  if (valid <= 0) {   // bought everything: any product but the positive
    if (I <= 1) {
      out_i[t] = p;
      return;
    }
    int64_t r = (int64_t)(u01(h, 0) * (float)(I - 1));
    if (r >= I - 1) r = I - 2;
    out_i[t] = r >= p ? r + 1 : r;
    return;
  }
  int64_t r = (int64_t)((double)u01(h, 0) * (double)valid);
  if (r >= valid) r = valid - 1;
  // the r-th id not in E = history U {p}: walk E in ascending order (merge p into the walk)
  int64_t x = r;
  bool p_done = p_in;
  for (int64_t e = h0; e < h1; ++e) {
    const int64_t v = hitem[e];
    if (!p_done && p < v) {
      if (p <= x) ++x;
      p_done = true;
    }
    if (v <= x) ++x;
    else if (p_done) break;
  }
  if (!p_done && p <= x) ++x;
  out_i[t] = x;
}

}  // namespace

// Vose's alias method on the host (one-time table construction; O(n)).  prob[i] in [0,1] and
// alias[i] such that P(i) = (prob[i] + sum_{j: alias[j] = i} (1 - prob[j])) / n = w[i] / sum(w).
extern "C" int ncf_alias_build(const double* weights, int64_t n, float* prob, int32_t* alias) {
  NCF_CHECK_ARG(n >= 1 && n < (int64_t)INT32_MAX, "ncf_alias_build: n out of range");
  double total = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    NCF_CHECK_ARG(weights[i] >= 0.0, "ncf_alias_build: negative weight");
    total += weights[i];
  }
  NCF_CHECK_ARG(total > 0.0, "ncf_alias_build: all weights are zero");
  std::vector<double> q(n);
  std::vector<int64_t> small, large;
  small.reserve(n);
  large.reserve(n);
  for (int64_t i = 0; i < n; ++i) {
    q[i] = weights[i] * (double)n / total;
    (q[i] < 1.0 ? small : large).push_back(i);
  }
  while (!small.empty() && !large.empty()) {
    const int64_t s = small.back(), l = large.back();
    small.pop_back();
    prob[s] = (float)q[s];
    alias[s] = (int32_t)l;
    q[l] = (q[l] + q[s]) - 1.0;
    if (q[l] < 1.0) {
      large.pop_back();
      small.push_back(l);
    }
  }
  for (int64_t i : large) { prob[i] = 1.0f; alias[i] = (int32_t)i; }
  for (int64_t i : small) { prob[i] = 1.0f; alias[i] = (int32_t)i; }   // rounding leftovers
  return NCF_OK;
}

extern "C" int ncf_sample_negatives(const int64_t* users, const int64_t* pos_items, int64_t batch,
                                    int64_t negatives, const float* alias_prob,
                                    const int32_t* alias_idx, int64_t n_items,
                                    const int64_t* hist_offsets, const int32_t* hist_items,
                                    int64_t n_users, uint64_t seed, int64_t max_attempts,
                                    int64_t* out_users, int64_t* out_items, float* out_targets,
                                    int* err_flag, void* stream) {
  NCF_CHECK_ARG(batch >= 0 && negatives >= 0 && n_items >= 1 && n_users >= 1 && max_attempts >= 0,
                "ncf_sample_negatives: bad sizes");
  NCF_CHECK_ARG(n_items < (int64_t)INT32_MAX, "ncf_sample_negatives: item ids must fit int32");
  const int64_t rows = batch * (negatives + 1);
  if (rows == 0) return NCF_OK;
  hipLaunchKernelGGL(k_negatives, dim3(ncf_cdiv(rows, 256)), dim3(256), 0, (hipStream_t)stream,
                     users, pos_items, batch, (int)negatives, alias_prob, alias_idx, n_items,
                     hist_offsets, hist_items, n_users, seed, (int)max_attempts, out_users,
                     out_items, out_targets, err_flag);
  NCF_CHECK_LAUNCH("ncf_sample_negatives");
  return NCF_OK;
}
