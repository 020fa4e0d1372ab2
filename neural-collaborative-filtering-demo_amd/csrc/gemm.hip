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

constexpr int BM = 64, BN = 64, BK = 32, LDP = 65;

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { F_RELU = 1, F_ACCUM = 2 };

// Per K-step each of the 256 threads stages 8 A and 8 B elements.  Index e = tid + 256*r maps
// to (row, k) with the CONTIGUOUS dimension on consecutive threads (coalesced loads); the
// k-major LDS image [BK][64+1] makes both the transposing writes and the MFMA operand reads
// (lane&31 -> row/col, lane>>5 -> k) bank-conflict-free.  The next K-step's global loads are
// issued into registers before the current step's MFMAs, so their latency hides under compute.
template <bool T_CONTIG_K>
__device__ __forceinline__ void tile_coord(int e, int& rc, int& k) {
  if (T_CONTIG_K) { k = e & (BK - 1); rc = e >> 5; }   // 32 consecutive k per row
  else { rc = e & 63; k = e >> 6; }                     // 64 consecutive rows per k
}

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

  float ra[8], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + 256 * r;
      int m, k;
      tile_coord<!A_T>(e, m, k);
      const int gm = m0 + m, gk = k0 + k;
      ra[r] = (gm < M && gk < ke) ? (A_T ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk]) : 0.0f;
      int n, k2;
      tile_coord<B_T>(e, n, k2);
      const int gn = n0 + n, gk2 = k0 + k2;
      rb[r] = (gn < N && gk2 < ke) ? (B_T ? B[(int64_t)gn * ldb + gk2] : B[(int64_t)gk2 * ldb + gn]) : 0.0f;
    }
  };
  if (kb < ke) load(kb);
  for (int k0 = kb; k0 < ke; k0 += BK) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + 256 * r;
      int m, k;
      tile_coord<!A_T>(e, m, k);
      As[k][m] = ra[r];
      int n, k2;
      tile_coord<B_T>(e, n, k2);
      Bs[k2][n] = rb[r];
    }
    __syncthreads();
    if (k0 + BK < ke) load(k0 + BK);  // prefetch next K-step; lands while the MFMAs run
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

// partial column sums: block (x = row chunk, y = 64-column chunk); waves stride the rows,
// lanes own columns (coalesced 256-B rows), 4-way unrolled; fixed-order LDS combine.
__global__ __launch_bounds__(256) void k_colsum_partial(const float* __restrict__ X, int64_t rows,
                                                        int64_t cols, int64_t ld,
                                                        int64_t rows_per_block,
                                                        float* __restrict__ part) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.y * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < cols) {
    int64_t r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      a0 += X[r * ld + c];
      a1 += X[(r + 4) * ld + c];
      a2 += X[(r + 8) * ld + c];
      a3 += X[(r + 12) * ld + c];
    }
    for (; r < r1; r += 4) a0 += X[r * ld + c];
  }
  red[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && c < cols)
    part[(int64_t)blockIdx.x * cols + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
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
  return (int64_t)splits * M * N + ncf_reduce_scratch(splits, M * N);
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
  if (workspace_floats < (int64_t)splits * M * N + ncf_reduce_scratch(splits, M * N)) {
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
  ncf_reduce_parts(workspace, K == 0 ? 1 : used, M * N, M * N, C, accumulate, N, ldc, st,
                   workspace + (int64_t)used * M * N);
  NCF_CHECK_LAUNCH("ncf_gemm_f32_splitk(reduce)");
  return NCF_OK;
}

static int64_t colsum_rpb(int64_t rows, int64_t cols) {
  // aim for ~512 blocks in total, at least 64 rows each
  const int64_t cb = (cols + 63) / 64;
  int64_t chunks = 512 / (cb > 0 ? cb : 1);
  if (chunks < 1) chunks = 1;
  int64_t rpb = (rows + chunks - 1) / chunks;
  return rpb < 64 ? 64 : rpb;
}

extern "C" int64_t ncf_colsum_workspace(int64_t rows, int64_t cols) {
  const int64_t rpb = colsum_rpb(rows, cols);
  const int64_t nb = (rows + rpb - 1) / rpb + 1;
  return nb * cols + ncf_reduce_scratch((int)nb, cols);
}

// out[c] (+)= sum_r X[r*ld + c]  (bias gradients), two deterministic passes
extern "C" int ncf_colsum(const float* X, int64_t rows, int64_t cols, int64_t ld, float* out,
                          int accumulate, float* workspace, int64_t workspace_floats,
                          void* stream) {
  NCF_CHECK_ARG(rows >= 0 && cols >= 0, "ncf_colsum: bad size");
  if (cols == 0) return NCF_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rpb = colsum_rpb(rows, cols);
  const int64_t nb = rows == 0 ? 1 : (rows + rpb - 1) / rpb;
  if (workspace_floats < ncf_colsum_workspace(rows, cols)) {
    ncf_set_error("ncf_colsum: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (rows == 0) {
    (void)hipMemsetAsync(workspace, 0, sizeof(float) * cols, st);
  } else {
    hipLaunchKernelGGL(k_colsum_partial, dim3((unsigned)nb, ncf_cdiv(cols, 64)), dim3(256), 0, st,
                       X, rows, cols, ld, rpb, workspace);
    NCF_CHECK_LAUNCH("ncf_colsum(partial)");
  }
  ncf_reduce_parts(workspace, (int)nb, cols, cols, out, accumulate, cols, cols, st,
                   workspace + nb * cols);
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
