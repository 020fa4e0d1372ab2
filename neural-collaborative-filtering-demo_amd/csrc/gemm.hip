// fp32 MFMA GEMM for the AdvancedNCF dense layers (attention Q/K/V/out projections and the MLP
// tower, src/model/architecture.py:27-30, :40-42, :57, :230-246) and their backward products.
//
// gfx950 has an exact f32-input matrix core: v_mfma_f32_32x32x2_f32 (64 FLOP/clk/SIMD, the f32
// vector rate, bit-for-bit a k-ordered fmaf chain).  The reference computes these layers in
// fp32, so fp32 MFMA keeps numerics at reference precision.
//
// Tiling: 256-thread workgroup = 4 waves, 64x64 output tile, each wave a 32x32 MFMA sub-tile with
// 16 accumulator registers per lane; BK = 16 staged through LDS as k-major [BK][64+1] images so
// the per-lane operand reads (lane&31 -> consecutive m/n, lane>>5 -> k) are conflict-free
// ds_read_b32 and the transposing writes hit 32 distinct banks.
//   A(i,k) = a_trans ? A[k*lda + i] : A[i*lda + k]
//   B(k,j) = b_trans ? B[j*ldb + k] : B[k*ldb + j]
// Weight gradients (reduction over the batch rows) use split-K slabs reduced in a fixed order,
// so results are bitwise reproducible run to run (no float atomics).
#include "ncf_common.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 16, LDP = 65;

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { F_RELU = 1, F_ACCUM = 2 };

template <bool A_T, bool B_T>
__global__ __launch_bounds__(256) void k_gemm_f32(int M, int N, int K, const float* __restrict__ A,
                                                  int64_t lda, const float* __restrict__ B,
                                                  int64_t ldb, float* __restrict__ C, int64_t ldc,
                                                  const float* __restrict__ bias, int flags,
                                                  int ksplit, int64_t c_split_stride) {
  __shared__ float As[BK][LDP];
  __shared__ float Bs[BK][LDP];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = blockIdx.z * ksplit;
  const int ke = min(K, kb + ksplit);
  C += (int64_t)blockIdx.z * c_split_stride;

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;

  for (int k0 = kb; k0 < ke; k0 += BK) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      int m, k;
      if (!A_T) { k = e & (BK - 1); m = e >> 4; } else { m = e & (BM - 1); k = e >> 6; }
      const int gm = m0 + m, gk = k0 + k;
      float v = 0.0f;
      if (gm < M && gk < ke) v = A_T ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk];
      As[k][m] = v;
      int n;
      if (B_T) { k = e & (BK - 1); n = e >> 4; } else { n = e & (BN - 1); k = e >> 6; }
      const int gn = n0 + n;
      const int gk2 = k0 + k;
      float u = 0.0f;
      if (gn < N && gk2 < ke) u = B_T ? B[(int64_t)gn * ldb + gk2] : B[(int64_t)gk2 * ldb + gn];
      Bs[k][n] = u;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[kk + (lane >> 5)][wm * 32 + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }

  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= N) return;
  const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < M) {
      float v = acc[r] + bv;
      if (flags & F_RELU) v = fmaxf(v, 0.0f);
      float* p = C + (int64_t)row * ldc + col;
      if (flags & F_ACCUM) v += *p;
      *p = v;
    }
  }
}

// out[i] (+)= sum_z part[z*stride + i], fixed z order
__global__ void k_sum_slabs(const float* __restrict__ part, int splits, int64_t stride, int64_t n,
                            float* __restrict__ out, int accumulate, int64_t rows, int64_t cols,
                            int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.0f;
  for (int z = 0; z < splits; ++z) s += part[z * stride + i];
  const int64_t r = i / cols, c = i % cols;
  float* p = out + r * ldo + c;
  *p = accumulate ? *p + s : s;
  (void)rows;
}

// partial column sums: part[b][c] = sum over rows [b*R, (b+1)*R) of X[r][c]
__global__ void k_colsum_partial(const float* __restrict__ X, int64_t rows, int64_t cols,
                                 int64_t ld, int64_t rows_per_block, float* __restrict__ part) {
  const int64_t c = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float s = 0.0f;
  for (int64_t r = r0; r < r1; ++r) s += X[r * ld + c];
  part[(int64_t)blockIdx.x * cols + c] = s;
}

template <bool A_T, bool B_T>
int launch(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
           int64_t ldb, float* C, int64_t ldc, const float* bias, int flags, int splits,
           int ksplit, int64_t c_split_stride, hipStream_t st) {
  dim3 grid(ncf_cdiv(M, BM), ncf_cdiv(N, BN), splits);
  hipLaunchKernelGGL((k_gemm_f32<A_T, B_T>), grid, dim3(256), 0, st, (int)M, (int)N, (int)K, A,
                     lda, B, ldb, C, ldc, bias, flags, ksplit, c_split_stride);
  NCF_CHECK_LAUNCH("ncf_gemm_f32");
  return NCF_OK;
}

int dispatch(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int a_trans,
             const float* B, int64_t ldb, int b_trans, float* C, int64_t ldc, const float* bias,
             int flags, int splits, int ksplit, int64_t c_split_stride, hipStream_t st) {
  if (!a_trans && !b_trans)
    return launch<false, false>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, st);
  if (!a_trans && b_trans)
    return launch<false, true>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, st);
  if (a_trans && !b_trans)
    return launch<true, false>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, st);
  return launch<true, true>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, st);
}

}  // namespace

// C[M,N] = act(A·B + bias) (flags bit0 relu; bit1 accumulate into C)
extern "C" int ncf_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                            int a_trans, const float* B, int64_t ldb, int b_trans, float* C,
                            int64_t ldc, const float* bias, int flags, void* stream) {
  NCF_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "ncf_gemm_f32: negative size");
  NCF_CHECK_ARG(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31), "ncf_gemm_f32: size too large");
  if (M == 0 || N == 0) return NCF_OK;
  NCF_CHECK_ARG(A && B && C, "ncf_gemm_f32: null pointer");
  return dispatch(M, N, K, A, lda, a_trans, B, ldb, b_trans, C, ldc, bias, flags, 1,
                  (int)((K + BK - 1) / BK * BK), 0, (hipStream_t)stream);
}

extern "C" int64_t ncf_gemm_splitk_workspace(int64_t M, int64_t N, int splits) {
  return (int64_t)splits * M * N;
}

// Long-K GEMM (weight gradients dW = dYᵀ·X, K = batch rows): K split into `splits` slabs, each a
// full [M,N] partial in `workspace`, summed in slab order into C (overwrite or accumulate).
extern "C" int ncf_gemm_f32_splitk(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                   int a_trans, const float* B, int64_t ldb, int b_trans, float* C,
                                   int64_t ldc, int accumulate, int splits, float* workspace,
                                   int64_t workspace_floats, void* stream) {
  NCF_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && splits >= 1, "ncf_gemm_f32_splitk: bad size");
  if (M == 0 || N == 0) return NCF_OK;
  NCF_CHECK_ARG(A && B && C && workspace, "ncf_gemm_f32_splitk: null pointer");
  if (workspace_floats < (int64_t)splits * M * N) {
    ncf_set_error("ncf_gemm_f32_splitk: workspace %lld < %lld floats", (long long)workspace_floats,
                  (long long)splits * M * N);
    return NCF_ERR_WORKSPACE;
  }
  int64_t ksplit = (K + splits - 1) / splits;
  ksplit = (ksplit + BK - 1) / BK * BK;
  const int used = (int)((K + ksplit - 1) / ksplit);
  hipStream_t st = (hipStream_t)stream;
  if (K == 0) {
    (void)hipMemsetAsync(workspace, 0, sizeof(float) * M * N, st);
  } else {
    int rc = dispatch(M, N, K, A, lda, a_trans, B, ldb, b_trans, workspace, N, nullptr, 0, used,
                      (int)ksplit, M * N, st);
    if (rc) return rc;
  }
  const int64_t n = M * N;
  hipLaunchKernelGGL(k_sum_slabs, dim3(ncf_cdiv(n, 256)), dim3(256), 0, st, workspace,
                     K == 0 ? 1 : used, M * N, n, C, accumulate, M, N, ldc);
  NCF_CHECK_LAUNCH("ncf_gemm_f32_splitk(reduce)");
  return NCF_OK;
}

extern "C" int64_t ncf_colsum_workspace(int64_t rows, int64_t cols) {
  const int64_t rpb = 256;
  return ((rows + rpb - 1) / rpb) * cols;
}

// out[c] (+)= sum_r X[r*ld + c]  (bias gradients), two deterministic passes
extern "C" int ncf_colsum(const float* X, int64_t rows, int64_t cols, int64_t ld, float* out,
                          int accumulate, float* workspace, int64_t workspace_floats,
                          void* stream) {
  NCF_CHECK_ARG(rows >= 0 && cols >= 0, "ncf_colsum: bad size");
  if (cols == 0) return NCF_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rpb = 256;
  const int64_t nb = rows == 0 ? 1 : (rows + rpb - 1) / rpb;
  if (workspace_floats < nb * cols) {
    ncf_set_error("ncf_colsum: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (rows == 0) {
    (void)hipMemsetAsync(workspace, 0, sizeof(float) * cols, st);
  } else {
    hipLaunchKernelGGL(k_colsum_partial, dim3((unsigned)nb, ncf_cdiv(cols, 256)), dim3(256), 0, st,
                       X, rows, cols, ld, rpb, workspace);
    NCF_CHECK_LAUNCH("ncf_colsum(partial)");
  }
  hipLaunchKernelGGL(k_sum_slabs, dim3(ncf_cdiv(cols, 256)), dim3(256), 0, st, workspace, (int)nb,
                     cols, cols, out, accumulate, (int64_t)1, cols, cols);
  NCF_CHECK_LAUNCH("ncf_colsum(reduce)");
  return NCF_OK;
}

namespace {
__global__ void k_fill_2d(float* __restrict__ p, int64_t rows, int64_t cols, int64_t ld, float v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  p[(i / cols) * ld + (i % cols)] = v;
}
}  // namespace

// p[r*ld + c] = value for r < rows, c < cols (e.g. the all-zero temporal columns of dW of mlp.0:
// the reference feeds zeros there, architecture.py:329-340, so their gradient is exactly 0)
extern "C" int ncf_fill_2d(float* p, int64_t rows, int64_t cols, int64_t ld, float value,
                           void* stream) {
  NCF_CHECK_ARG(rows >= 0 && cols >= 0 && ld >= cols, "ncf_fill_2d: bad shape");
  if (rows == 0 || cols == 0) return NCF_OK;
  hipLaunchKernelGGL(k_fill_2d, dim3(ncf_cdiv(rows * cols, 256)), dim3(256), 0,
                     (hipStream_t)stream, p, rows, cols, ld, value);
  NCF_CHECK_LAUNCH("ncf_fill_2d");
  return NCF_OK;
}
