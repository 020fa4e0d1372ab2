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

// 128x64 output tile per 256-thread workgroup (4 waves as 2x2, each wave 64x32 = two 32x32
// MFMA accumulators sharing one B fragment), BK = 32 staged through LDS as k-major images.
// Global loads are float4 along whichever dimension is contiguous in memory (coalesced), the
// next K-step is prefetched into registers while the current one runs on the matrix cores.
constexpr int BM = 128, BN = 64, BK = 32;

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { F_RELU = 1, F_ACCUM = 2 };

// guarded float4 load of up to 4 consecutive elements (count = valid elements)
__device__ __forceinline__ float4 ld4_guard(const float* p, int count, bool vec) {
  if (count >= 4 && vec) return ld4(p);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (count > 0) v.x = p[0];
  if (count > 1) v.y = p[1];
  if (count > 2) v.z = p[2];
  if (count > 3) v.w = p[3];
  return v;
}

template <bool A_T, bool B_T>
__global__ __launch_bounds__(256) void k_gemm_f32(int M, int N, int K, const float* __restrict__ A,
                                                  int64_t lda, const float* __restrict__ B,
                                                  int64_t ldb, float* __restrict__ C, int64_t ldc,
                                                  const float* __restrict__ bias, int flags,
                                                  int ksplit, int64_t c_split_stride, int vec,
                                                  float* __restrict__ rowsum_part) {
  // k-major LDS images; row pitch padded (+1 for transposing scalar writes, +4 for b128 writes)
  constexpr int LDA = A_T ? BM + 4 : BM + 1;
  constexpr int LDB = B_T ? BN + 1 : BN + 4;
  __shared__ __attribute__((aligned(16))) float As[BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[BK * LDB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = blockIdx.z * ksplit;
  const int ke = min(K, kb + ksplit);
  C += (int64_t)blockIdx.z * c_split_stride;

  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { acc0[r] = 0.0f; acc1[r] = 0.0f; }
  // row sums of A over this block's K range (bias gradient when A = dYᵀ): column-0 blocks only
  const bool do_rs = rowsum_part != nullptr && blockIdx.y == 0 && tid < BM;
  float rs = 0.0f;

  float4 ra[4], rb[2];
  // interior tiles (block-uniform test) take unguarded float4 loads: no exec-masked branches
  // around the prefetch, so the compiler keeps it in flight across the MFMAs
  const bool interior = vec && m0 + BM <= M && n0 + BN <= N;
  auto load = [&](int k0) {
    if (interior && k0 + BK <= ke) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = tid + 256 * r;
        ra[r] = !A_T ? ld4(A + (int64_t)(m0 + (e >> 3)) * lda + k0 + (e & 7) * 4)
                     : ld4(A + (int64_t)(k0 + (e >> 5)) * lda + m0 + (e & 31) * 4);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int e = tid + 256 * r;
        rb[r] = B_T ? ld4(B + (int64_t)(n0 + (e >> 3)) * ldb + k0 + (e & 7) * 4)
                    : ld4(B + (int64_t)(k0 + (e >> 4)) * ldb + n0 + (e & 15) * 4);
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      if (!A_T) {  // A[m][k], k contiguous
        const int m = e >> 3, k4 = (e & 7) * 4;
        const int gm = m0 + m, gk = k0 + k4;
        ra[r] = gm < M ? ld4_guard(A + (int64_t)gm * lda + gk, ke - gk, vec) : make_float4(0, 0, 0, 0);
      } else {     // A[k][m], m contiguous
        const int m4 = (e & 31) * 4, k = e >> 5;
        const int gm = m0 + m4, gk = k0 + k;
        ra[r] = gk < ke ? ld4_guard(A + (int64_t)gk * lda + gm, M - gm, vec) : make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int e = tid + 256 * r;
      if (B_T) {   // B[n][k], k contiguous
        const int n = e >> 3, k4 = (e & 7) * 4;
        const int gn = n0 + n, gk = k0 + k4;
        rb[r] = gn < N ? ld4_guard(B + (int64_t)gn * ldb + gk, ke - gk, vec) : make_float4(0, 0, 0, 0);
      } else {     // B[k][n], n contiguous
        const int n4 = (e & 15) * 4, k = e >> 4;
        const int gn = n0 + n4, gk = k0 + k;
        rb[r] = gk < ke ? ld4_guard(B + (int64_t)gk * ldb + gn, N - gn, vec) : make_float4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      if (!A_T) {
        const int m = e >> 3, k4 = (e & 7) * 4;
        As[(k4 + 0) * LDA + m] = ra[r].x; As[(k4 + 1) * LDA + m] = ra[r].y;
        As[(k4 + 2) * LDA + m] = ra[r].z; As[(k4 + 3) * LDA + m] = ra[r].w;
      } else {
        const int m4 = (e & 31) * 4, k = e >> 5;
        *reinterpret_cast<float4*>(&As[k * LDA + m4]) = ra[r];
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int e = tid + 256 * r;
      if (B_T) {
        const int n = e >> 3, k4 = (e & 7) * 4;
        Bs[(k4 + 0) * LDB + n] = rb[r].x; Bs[(k4 + 1) * LDB + n] = rb[r].y;
        Bs[(k4 + 2) * LDB + n] = rb[r].z; Bs[(k4 + 3) * LDB + n] = rb[r].w;
      } else {
        const int n4 = (e & 15) * 4, k = e >> 4;
        *reinterpret_cast<float4*>(&Bs[k * LDB + n4]) = rb[r];
      }
    }
  };
  if (kb < ke) load(kb);
  for (int k0 = kb; k0 < ke; k0 += BK) {
    store();
    __syncthreads();
    if (k0 + BK < ke) load(k0 + BK);  // next K-step lands while the MFMAs run
    if (do_rs) {
#pragma unroll
      for (int k = 0; k < BK; ++k) rs += As[k * LDA + tid];
    }
    // read every fragment of the K-step first (one LDS round trip), then 32 back-to-back MFMAs
    float fa0[BK / 2], fa1[BK / 2], fb[BK / 2];
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int k = 2 * kk + (lane >> 5);
      fa0[kk] = As[k * LDA + wm * 64 + (lane & 31)];
      fa1[kk] = As[k * LDA + wm * 64 + 32 + (lane & 31)];
      fb[kk] = Bs[k * LDB + wn * 32 + (lane & 31)];
    }
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa0[kk], fb[kk], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa1[kk], fb[kk], acc1, 0, 0, 0);
    }
    __syncthreads();
  }

  if (do_rs && m0 + tid < M) rowsum_part[(int64_t)blockIdx.z * M + m0 + tid] = rs;
  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= N) return;
  const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * 64 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) {
        float v = (t ? acc1[r] : acc0[r]) + bv;
        if (flags & F_RELU) v = fmaxf(v, 0.0f);
        float* p = C + (int64_t)row * ldc + col;
        if (flags & F_ACCUM) v += *p;
        *p = v;
      }
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
           int ksplit, int64_t c_split_stride, float* rowsum, hipStream_t st) {
  const int vec = (lda % 4 == 0) && (ldb % 4 == 0) && ((uintptr_t)A % 16 == 0) &&
                  ((uintptr_t)B % 16 == 0) && (ksplit % 4 == 0);
  dim3 grid(ncf_cdiv(M, BM), ncf_cdiv(N, BN), splits);
  hipLaunchKernelGGL((k_gemm_f32<A_T, B_T>), grid, dim3(256), 0, st, (int)M, (int)N, (int)K, A,
                     lda, B, ldb, C, ldc, bias, flags, ksplit, c_split_stride, vec, rowsum);
  NCF_CHECK_LAUNCH("ncf_gemm_f32");
  return NCF_OK;
}

int dispatch(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int a_trans,
             const float* B, int64_t ldb, int b_trans, float* C, int64_t ldc, const float* bias,
             int flags, int splits, int ksplit, int64_t c_split_stride, hipStream_t st,
             float* rowsum = nullptr) {
  if (!a_trans && !b_trans)
    return launch<false, false>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, rowsum, st);
  if (!a_trans && b_trans)
    return launch<false, true>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, rowsum, st);
  if (a_trans && !b_trans)
    return launch<true, false>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, rowsum, st);
  return launch<true, true>(M, N, K, A, lda, B, ldb, C, ldc, bias, flags, splits, ksplit, c_split_stride, rowsum, st);
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
  return (int64_t)splits * (M * N + M) + ncf_reduce_scratch(splits, M * N);
}

// Long-K GEMM (weight gradients dW = dYᵀ·X, K = batch rows): K split into `splits` slabs, each a
// full [M,N] partial in `workspace` (+ a [M] row-sum partial when row_sums != NULL), summed in
// slab order into C (overwrite or accumulate) — inline, or appended to `defer`.
extern "C" int ncf_gemm_f32_splitk(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                   int a_trans, const float* B, int64_t ldb, int b_trans, float* C,
                                   int64_t ldc, int accumulate, float* row_sums, int splits,
                                   float* workspace, int64_t workspace_floats,
                                   ncf_reduce_list* defer, void* stream) {
  NCF_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && splits >= 1, "ncf_gemm_f32_splitk: bad size");
  NCF_CHECK_ARG(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31) && M * N < (1ll << 31),
                "ncf_gemm_f32_splitk: size too large");
  if (M == 0 || N == 0) return NCF_OK;
  NCF_CHECK_ARG(A && B && C && workspace, "ncf_gemm_f32_splitk: null pointer");
  if (workspace_floats < ncf_gemm_splitk_workspace(M, N, splits)) {
    ncf_set_error("ncf_gemm_f32_splitk: workspace %lld < %lld floats", (long long)workspace_floats,
                  (long long)ncf_gemm_splitk_workspace(M, N, splits));
    return NCF_ERR_WORKSPACE;
  }
  int64_t ksplit = (K + splits - 1) / splits;
  ksplit = (ksplit + BK - 1) / BK * BK;
  if (ksplit == 0) ksplit = BK;
  const int used = K == 0 ? 1 : (int)((K + ksplit - 1) / ksplit);
  hipStream_t st = (hipStream_t)stream;
  float* slabs = workspace;
  float* rsp = workspace + (int64_t)splits * M * N;   // [used][M] row-sum partials
  float* scratch = rsp + (int64_t)splits * M;
  if (K == 0) {
    (void)hipMemsetAsync(slabs, 0, sizeof(float) * M * N, st);
    if (row_sums) (void)hipMemsetAsync(rsp, 0, sizeof(float) * M, st);
  } else {
    int rc = dispatch(M, N, K, A, lda, a_trans, B, ldb, b_trans, slabs, N, nullptr, 0, used,
                      (int)ksplit, M * N, st, row_sums ? rsp : nullptr);
    if (rc) return rc;
  }
  if (defer) {
    int rc = ncf_defer(defer, slabs, used, M * N, M * N, C, accumulate, N, ldc);
    if (!rc && row_sums) rc = ncf_defer(defer, rsp, used, M, M, row_sums, 0, M, M);
    return rc;
  }
  ncf_reduce_parts(slabs, used, M * N, M * N, C, accumulate, N, ldc, st, scratch);
  if (row_sums) ncf_reduce_parts(rsp, used, M, M, row_sums, 0, M, M, st, scratch);
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
