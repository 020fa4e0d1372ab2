// Weights-resident streaming GEMM for the tall-skinny AdvancedNCF layers: C[M,N] = act(A[M,K]·B + b)
// with M = batch rows (20480 at C2) and K, N <= 256 — the MLP tower (src/model/architecture.py
// :230-246) and the attention projections (:40-42, :57), forward and dX.
//
// The whole B operand (N x K fp32, <= 132 KB) is staged ONCE per workgroup into LDS as an
// [N][K+1] image; the workgroup then streams 32-row tiles of A: N/64 waves share a tile, each
// owning 64 output columns (two v_mfma_f32_32x32x2_f32 accumulators), so a row tile completes
// inside one workgroup and no per-K-step barrier exists.
//   A fragments: MFMA step s of a 64-deep k chunk uses k = s + 32h for lane half h, so a lane's A
//                operand is a 32-float contiguous run of its row (8 float4 loads, the next chunk
//                prefetched while the current one multiplies);
//   B fragments: LDS reads Bs[j][kc + s + 32h], j = lane&31 + 32t: bank (j + k) mod 64 -> the 64
//                lanes hit 64 distinct banks (the +1 pitch).
// Full output rows live in one workgroup, so row-wise epilogues (LayerNorm) can fuse here.
#include "ncf_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { F_RELU = 1, F_ACCUM = 2 };

template <int K, int N>
struct RowsGeo {
  // a workgroup owns NB output columns (grid.y = N / NB): <= ~66 KB of LDS so >= 2 workgroups
  // (8 waves) share a CU
  static constexpr int NB = (K <= 128 && N >= 128) ? 128 : 64;
  static constexpr int WPT = NB / 64;        // waves per 32-row tile (64 output columns each)
  static constexpr int NT = 2;               // 32x32 accumulator tiles per wave
  static constexpr int KC = K / 64;          // 64-deep k chunks
  static constexpr int PITCH = K + 1;
  static constexpr int LDS_FLOATS = NB * PITCH;
};

// B(k, j) = b_trans ? B[j*ldb + k] : B[k*ldb + j]
template <int K, int N>
__device__ __forceinline__ void stage_b(float* Bs, const float* __restrict__ B, int64_t ldb,
                                        int b_trans) {
  using G = RowsGeo<K, N>;
  constexpr int NB = G::NB;
  if (b_trans) {  // rows j of B are contiguous in k: float4 reads
    for (int e = threadIdx.x; e < NB * (K / 4); e += blockDim.x) {
      const int j = e / (K / 4), k4 = (e % (K / 4)) * 4;
      const float4 v = ld4(B + (int64_t)j * ldb + k4);
      float* d = Bs + j * G::PITCH + k4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  } else {        // rows k of B are contiguous in j
    for (int e = threadIdx.x; e < K * (NB / 4); e += blockDim.x) {
      const int k = e / (NB / 4), j4 = (e % (NB / 4)) * 4;
      const float4 v = ld4(B + (int64_t)k * ldb + j4);
      Bs[(j4 + 0) * G::PITCH + k] = v.x;
      Bs[(j4 + 1) * G::PITCH + k] = v.y;
      Bs[(j4 + 2) * G::PITCH + k] = v.z;
      Bs[(j4 + 3) * G::PITCH + k] = v.w;
    }
  }
}

template <int K, int N>
__global__ __launch_bounds__(256) void k_gemm_rows(int M, const float* __restrict__ A, int64_t lda,
                                                   const float* __restrict__ B, int64_t ldb,
                                                   int b_trans, float* __restrict__ C, int64_t ldc,
                                                   const float* __restrict__ bias, int flags) {
  using G = RowsGeo<K, N>;
  extern __shared__ __attribute__((aligned(16))) float Bs[];
  const int n0 = blockIdx.y * G::NB;         // this workgroup's output columns
  stage_b<K, N>(Bs, b_trans ? B + (int64_t)n0 * ldb : B + n0, ldb, b_trans);
  C += n0;
  if (bias) bias += n0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int tiles = (M + 31) / 32;
  const int wc = w % G::WPT;                 // this wave's 64-column slice
  constexpr int TPB = 4 / G::WPT;            // row tiles per block iteration
  float bv[G::NT];
#pragma unroll
  for (int t = 0; t < G::NT; ++t) bv[t] = bias ? bias[wc * 64 + t * 32 + i] : 0.0f;
  const float* bw = Bs + (wc * 64 + i) * G::PITCH + 32 * h;
  for (int tile = blockIdx.x * TPB + w / G::WPT; tile < tiles; tile += gridDim.x * TPB) {
    const int row0 = tile * 32;
    const float* ap = A + (int64_t)(row0 + i < M ? row0 + i : 0) * lda + 32 * h;
    f32x16 acc[G::NT];
#pragma unroll
    for (int t = 0; t < G::NT; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.0f;
    // Loads are unconditional (rows past M read row 0; their outputs are never stored, and MFMA
    // rows are independent): no exec-masked branches, so the prefetch really overlaps — a
    // guarded load makes the compiler wait vmcnt(0) on the prefetch it just issued.
    float4 a[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] = ld4(ap + 4 * q);
#pragma unroll 1
    for (int kc = 0; kc < G::KC; ++kc) {
      const int kn = kc + 1 < G::KC ? kc + 1 : kc;  // last chunk re-reads itself (no branch)
      float4 an[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) an[q] = ld4(ap + kn * 64 + 4 * q);
      // keep the 8 prefetch loads here (the scheduler would otherwise sink each load next to
      // its use in the next chunk and expose its full latency)
      __builtin_amdgcn_sched_barrier(0);
      const float* bk = bw + kc * 64;
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        const float4 v4 = a[s >> 2];
        const float av = (s & 3) == 0 ? v4.x : (s & 3) == 1 ? v4.y : (s & 3) == 2 ? v4.z : v4.w;
#pragma unroll
        for (int t = 0; t < G::NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bk[t * 32 * G::PITCH + s], acc[t], 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = an[q];
    }
    // epilogue: C row = row0 + (r&3) + 8(r>>2) + 4h, col = 64wc + 32t + i
#pragma unroll
    for (int t = 0; t < G::NT; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < M) {
          float v = acc[t][r] + bv[t];
          if (flags & F_RELU) v = fmaxf(v, 0.0f);
          float* p = C + (int64_t)row * ldc + wc * 64 + t * 32 + i;
          if (flags & F_ACCUM) v += *p;
          *p = v;
        }
      }
    }
  }
}

int g_cus = 0;

template <int K, int N>
int launch_rows(int64_t M, const float* A, int64_t lda, const float* B, int64_t ldb, int b_trans,
                float* C, int64_t ldc, const float* bias, int flags, hipStream_t st) {
  using G = RowsGeo<K, N>;
  const size_t lds = sizeof(float) * G::LDS_FLOATS;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_gemm_rows<K, N>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  if (g_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  const int per_cu = (int)(160 * 1024 / (lds + 1024));
  const int64_t tiles = (M + 31) / 32;
  int64_t grid = (int64_t)g_cus * (per_cu > 0 ? (per_cu > 4 ? 4 : per_cu) : 1) / (N / G::NB);
  if (grid < g_cus / 2) grid = g_cus / 2;
  const int64_t need = (tiles + (4 / G::WPT) - 1) / (4 / G::WPT);
  if (grid > need) grid = need;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((k_gemm_rows<K, N>), dim3((unsigned)grid, N / G::NB), dim3(256), lds, st, (int)M, A, lda,
                     B, ldb, b_trans, C, ldc, bias, flags);
  NCF_CHECK_LAUNCH("ncf_gemm_rows");
  return NCF_OK;
}

}  // namespace

// C[M,N] = act(A·B + bias) for row-major A [M,K] (a_trans = 0 only), K, N in {64, 128, 256};
// same B / flags convention as ncf_gemm_f32.
extern "C" int ncf_gemm_rows(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                             const float* B, int64_t ldb, int b_trans, float* C, int64_t ldc,
                             const float* bias, int flags, void* stream) {
  NCF_CHECK_ARG(M >= 0 && M < (1ll << 31), "ncf_gemm_rows: bad M");
  NCF_CHECK_ARG(A && B && C, "ncf_gemm_rows: null pointer");
  NCF_CHECK_ARG(lda % 4 == 0 && ((uintptr_t)A) % 16 == 0 && ldb % 4 == 0 &&
                    ((uintptr_t)B) % 16 == 0,
                "ncf_gemm_rows: A/B must be 16-byte aligned with ld %% 4 == 0");
  if (M == 0) return NCF_OK;
  hipStream_t st = (hipStream_t)stream;
#define NCF_ROWS(KK, NN) \
  if (K == KK && N == NN) return launch_rows<KK, NN>(M, A, lda, B, ldb, b_trans, C, ldc, bias, flags, st);
  NCF_ROWS(64, 64) NCF_ROWS(64, 128) NCF_ROWS(64, 256)
  NCF_ROWS(128, 64) NCF_ROWS(128, 128) NCF_ROWS(128, 256)
  NCF_ROWS(256, 64) NCF_ROWS(256, 128)
#undef NCF_ROWS
  ncf_set_error("ncf_gemm_rows: unsupported (K=%lld, N=%lld)", (long long)K, (long long)N);
  return NCF_ERR_ARG;
}
