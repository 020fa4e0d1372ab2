// LDS-free fp32 MFMA GEMM for the tall-skinny AdvancedNCF layers (M = batch rows, N, K <= 256).
//
// One wave owns a 32x32 output tile and feeds v_mfma_f32_32x32x2_f32 straight from global
// memory.  The trick is the k order: MFMA step s of a 64-deep k-chunk uses k = s + 32h for lane
// half h (the sum over k does not care about the order, both operands just have to agree).  Then
//   * an operand stored with k CONTIGUOUS (row-major X[M,K], or W[N,K] read as Wᵀ) is a run of
//     32 consecutive floats per lane: 8 float4 loads, all in flight before the 32 MFMAs;
//   * an operand stored with k STRIDED (dY read as dYᵀ, W[N,K] read as W) is, at each step, one
//     float per lane with lanes 0-31 on 32 consecutive floats of one row: fully coalesced.
// No LDS, no barriers; the 4 waves of a block are independent tasks.  (The kernel also supports
// K slabs and A row sums; the weight gradients use the LDS-tiled split-K kernel of gemm.hip,
// which measured faster at the C2 shapes — tools/gemm_bench.py.)
//
// Reference layers: attention projections (src/model/architecture.py:40-42, :57) and the MLP
// tower (:230-246), forward and backward.
#include "ncf_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { F_RELU = 1, F_ACCUM = 2 };

// CONTIG: element (r, k) at base[r*ld + k]; STRIDE: element (r, k) at base[k*ld + r]
template <bool CONTIG>
struct Opnd {
  const float* base;
  int64_t ld;
  int R;  // rows of the operand in its own index (M for A, N for B)
};

template <bool A_CONTIG, bool B_CONTIG>
__global__ __launch_bounds__(256) void k_gemm_direct(
    int M, int N, int K, const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
    int64_t ldb, float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, int flags,
    int ksplit, int64_t c_split_stride, float* __restrict__ colsum_part, int vec_ok) {
  const int lane = threadIdx.x & 63;
  const int task = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int tm = (M + 31) / 32, tn = (N + 31) / 32;
  if (task >= tm * tn) return;  // whole wave retires
  const int ti = task / tn, tj = task % tn;
  const int i0 = ti * 32, j0 = tj * 32;
  const int r = lane & 31, h = lane >> 5;
  const int kb = blockIdx.y * ksplit;
  const int ke = min(K, kb + ksplit);
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
  float csum = 0.0f;  // column sum of A over k (bias gradient), lanes of this tile
  const int ia = i0 + r, jb = j0 + r;
  const bool a_in = ia < M, b_in = jb < N;
  for (int kc = kb; kc < ke; kc += 64) {
    const bool full = kc + 64 <= ke;
    float a[32], b[32];
    // ---- operand A: a[s] = A(ia, kc + s + 32h)
    if (A_CONTIG) {
      const float* p = A + (int64_t)ia * lda + kc + 32 * h;
      if (full && vec_ok && a_in) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float4 v = ld4(p + 4 * q);
          a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int s = 0; s < 32; ++s) a[s] = (a_in && kc + s + 32 * h < ke) ? p[s] : 0.0f;
      }
    } else {
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        const int k = kc + s + 32 * h;
        a[s] = (a_in && k < ke) ? A[(int64_t)k * lda + ia] : 0.0f;
      }
    }
    // ---- operand B: b[s] = B(kc + s + 32h, jb)
    if (B_CONTIG) {
      const float* p = B + (int64_t)jb * ldb + kc + 32 * h;
      if (full && vec_ok && b_in) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float4 v = ld4(p + 4 * q);
          b[4 * q] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int s = 0; s < 32; ++s) b[s] = (b_in && kc + s + 32 * h < ke) ? p[s] : 0.0f;
      }
    } else {
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        const int k = kc + s + 32 * h;
        b[s] = (b_in && k < ke) ? B[(int64_t)k * ldb + jb] : 0.0f;
      }
    }
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
    if (colsum_part && tj == 0) {
#pragma unroll
      for (int s = 0; s < 32; ++s) csum += a[s];
    }
  }
  if (colsum_part && tj == 0) {
    csum += __shfl_xor(csum, 32, 64);
    if (h == 0 && a_in) colsum_part[(int64_t)blockIdx.y * M + ia] = csum;
  }
  C += (int64_t)blockIdx.y * c_split_stride;
  const int col = j0 + r;
  if (col >= N) return;
  const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int row = i0 + (q & 3) + 8 * (q >> 2) + 4 * h;
    if (row < M) {
      float v = acc[q] + bv;
      if (flags & F_RELU) v = fmaxf(v, 0.0f);
      float* p = C + (int64_t)row * ldc + col;
      if (flags & F_ACCUM) v += *p;
      *p = v;
    }
  }
}

template <bool AC, bool BC>
void launch(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
            int64_t ldb, float* C, int64_t ldc, const float* bias, int flags, int splits,
            int ksplit, int64_t cstride, float* colsum, int vec_ok, hipStream_t st) {
  const int64_t tasks = ((M + 31) / 32) * ((N + 31) / 32);
  hipLaunchKernelGGL((k_gemm_direct<AC, BC>), dim3(ncf_cdiv(tasks, 4), splits), dim3(256), 0, st,
                     (int)M, (int)N, (int)K, A, lda, B, ldb, C, ldc, bias, flags, ksplit, cstride,
                     colsum, vec_ok);
}

int dispatch(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int a_trans,
             const float* B, int64_t ldb, int b_trans, float* C, int64_t ldc, const float* bias,
             int flags, int splits, int ksplit, int64_t cstride, float* colsum, hipStream_t st) {
  // CONTIG A <=> A row-major [M,K] (a_trans == 0); CONTIG B <=> B stored [N,K] (b_trans == 1)
  const bool ac = !a_trans, bc = b_trans;
  const int vec_ok = ((ac ? lda : 4) % 4 == 0) && ((bc ? ldb : 4) % 4 == 0) &&
                     (((uintptr_t)A) % 16 == 0) && (((uintptr_t)B) % 16 == 0) &&
                     (ksplit % 64 == 0);
  if (ac && bc) launch<true, true>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, cstride, colsum, vec_ok, st);
  else if (ac) launch<true, false>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, cstride, colsum, vec_ok, st);
  else if (bc) launch<false, true>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, cstride, colsum, vec_ok, st);
  else launch<false, false>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, cstride, colsum, vec_ok, st);
  NCF_CHECK_LAUNCH("ncf_gemm_direct");
  return NCF_OK;
}

}  // namespace

// C[M,N] = act(A·B + bias), same operand convention as ncf_gemm_f32 (include/ncf_hip.h).
extern "C" int ncf_gemm_direct(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                               int a_trans, const float* B, int64_t ldb, int b_trans, float* C,
                               int64_t ldc, const float* bias, int flags, void* stream) {
  NCF_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31),
                "ncf_gemm_direct: bad size");
  if (M == 0 || N == 0) return NCF_OK;
  NCF_CHECK_ARG(A && B && C, "ncf_gemm_direct: null pointer");
  const int64_t kpad = (K + 63) / 64 * 64;
  return dispatch(M, N, K, A, lda, a_trans, B, ldb, b_trans, C, ldc, bias, flags, 1,
                  (int)(kpad > 0 ? kpad : 64), 0, nullptr, (hipStream_t)stream);
}
