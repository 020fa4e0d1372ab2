// Standalone A/B bench of the deferred-Adam rolling sweep (GPU box only; not part of the library).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<csrc> -I<include> tools/sweep_bench.hip -o sweep_bench
//   ./sweep_bench
//
// The library's adam.hip is compiled into this translation unit, so the variants below call the
// very same adam0 replay.  C2 geometry: users 1M x 64 and items 100K x 64, GMF + MLP pair per id
// kind, sweep_every 64.  Stamps: a steady-state mix (3/4 of the rows owe the full 64 steps, the
// rest a uniform 1..63).  Every variant starts from the same state and must leave bit-identical
// p/m/v/stamp to the library kernel; the time is the mean of 50 launches (HIP events).
#include "../neural-collaborative-filtering-demo_amd/csrc/capi.hip"
#include "../neural-collaborative-filtering-demo_amd/csrc/adam.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

namespace {

// V1: persistent waves over a flattened (kind, row) space with the next row's p/m/v loaded
// before the current row's replay (one row of both tables of a pair per wave, D = 64).
template <int D>
__global__ __launch_bounds__(256) void k_sweep_v1(const PairArgs a, int32_t every, int32_t step_rel,
                                                  const ncf_step_clock* __restrict__ clock,
                                                  const float* __restrict__ table, AdamScalars s) {
  static_assert(D == 64, "v1: one row per wave");
  const int32_t target = clock->t + step_rel;
  int64_t row0[2], nrow[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t slice = (a.rows[k] + every - 1) / every;
    row0[k] = (int64_t)(target % every) * slice;
    nrow[k] = max((int64_t)0, min(slice, a.rows[k] - row0[k]));
  }
  const int64_t total = nrow[0] + nrow[1];
  const int lane = threadIdx.x & 63;
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  auto locate = [&](int64_t e, int& k, int64_t& row) {
    k = e < nrow[0] ? 0 : 1;
    row = row0[k] + (k ? e - nrow[0] : e);
  };
  int64_t e = wv;
  if (e >= total) return;
  int k;
  int64_t row;
  locate(e, k, row);
  float p0, m0, v0, p1, m1, v1;
  int32_t from;
  {
    const TablePtrs& t = a.t[k];
    const int64_t o = row * D + lane;
    p0 = t.p0[o]; m0 = t.m0[o]; v0 = t.v0[o]; p1 = t.p1[o]; m1 = t.m1[o]; v1 = t.v1[o];
    from = a.stamp[k][row];
  }
  while (true) {
    const int64_t en = e + nw;
    int kn = 0;
    int64_t rown = 0;
    float np0 = 0.f, nm0 = 0.f, nv0 = 0.f, np1 = 0.f, nm1 = 0.f, nv1 = 0.f;
    int32_t nfrom = 0;
    const bool more = en < total;
    if (more) {
      locate(en, kn, rown);
      const TablePtrs& t = a.t[kn];
      const int64_t o = rown * D + lane;
      np0 = t.p0[o]; nm0 = t.m0[o]; nv0 = t.v0[o]; np1 = t.p1[o]; nm1 = t.m1[o]; nv1 = t.v1[o];
      nfrom = a.stamp[kn][rown];
    }
    const int32_t f = __builtin_amdgcn_readfirstlane(from);
    if (f < target) {
      replay_uniform<1, true>(&p0, &m0, &v0, &p1, &m1, &v1, f, target, table, s);
      const TablePtrs& t = a.t[k];
      const int64_t o = row * D + lane;
      t.p0[o] = p0; t.m0[o] = m0; t.v0[o] = v0; t.p1[o] = p1; t.m1[o] = m1; t.v1[o] = v1;
      if (lane == 0) a.stamp[k][row] = target;
    }
    if (!more) break;
    e = en; k = kn; row = rown;
    p0 = np0; m0 = nm0; v0 = nv0; p1 = np1; m1 = nm1; v1 = nv1; from = nfrom;
  }
}

// V2: the library kernel's body over a flattened (kind, row) grid (no idle item blocks)
template <int D>
__global__ __launch_bounds__(256) void k_sweep_v2(const PairArgs a, int32_t every, int32_t step_rel,
                                                  const ncf_step_clock* __restrict__ clock,
                                                  const float* __restrict__ table, AdamScalars s) {
  constexpr int L = Replay<D>::LPR;
  const int32_t target = clock->t + step_rel;
  int64_t row0[2], nrow[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t slice = (a.rows[k] + every - 1) / every;
    row0[k] = (int64_t)(target % every) * slice;
    nrow[k] = max((int64_t)0, min(slice, a.rows[k] - row0[k]));
  }
  const int64_t n = (nrow[0] + nrow[1]) * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / L;
    const int k = r < nrow[0] ? 0 : 1;
    const int64_t row = row0[k] + (k ? r - nrow[0] : r);
    const int sub = (int)(e % L);
    int32_t* stamp = a.stamp[k];
    const int32_t from = stamp[row];
    catch_up_row<D, false>(a.t[k], row, sub, from, target, table, s);
    if (sub == 0 && from < target) stamp[row] = target;
  }
}

// V3: RPW rows (pairs) per wave, LPR = 64 / RPW lanes per row, EPL = RPW columns per lane: RPW x
// more independent replay chains per lane.  The rows' owed ranges differ: steps every row of the
// wave owes run unmasked (chunked scalar step scalars, replay_uniform); the steps before that run
// under a per-lane predicate.
template <int RPW>
__global__ __launch_bounds__(256) void k_sweep_v3(const PairArgs a, int32_t every, int32_t step_rel,
                                                  const ncf_step_clock* __restrict__ clock,
                                                  const float* __restrict__ table, AdamScalars s) {
  constexpr int D = 64, LPR = 64 / RPW, EPL = RPW;
  const int32_t target = clock->t + step_rel;
  int64_t row0[2], nrow[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t slice = (a.rows[k] + every - 1) / every;
    row0[k] = (int64_t)(target % every) * slice;
    nrow[k] = max((int64_t)0, min(slice, a.rows[k] - row0[k]));
  }
  const int64_t total = nrow[0] + nrow[1];
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wv; w * RPW < total; w += nw) {
    const int64_t e = w * RPW + lane / LPR;
    const bool valid = e < total;
    const int k = e < nrow[0] ? 0 : 1;
    const int64_t row = valid ? row0[k] + (k ? e - nrow[0] : e) : 0;
    const TablePtrs& t = a.t[k];
    const int32_t from = valid ? a.stamp[k][row] : target;
    const int32_t fe = min(from, target);   // locked / current rows: nothing owed
    int32_t fmin = fe, fmax = fe;
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) {
      fmin = min(fmin, __shfl_xor(fmin, o, 64));
      fmax = max(fmax, __shfl_xor(fmax, o, 64));
    }
    fmin = __builtin_amdgcn_readfirstlane(fmin);
    fmax = __builtin_amdgcn_readfirstlane(fmax);
    if (fmin >= target) continue;
    const int64_t o = row * D + sub;
    float p0[EPL], m0[EPL], v0[EPL], p1[EPL], m1[EPL], v1[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      p0[j] = t.p0[o + j * LPR]; m0[j] = t.m0[o + j * LPR]; v0[j] = t.v0[o + j * LPR];
      p1[j] = t.p1[o + j * LPR]; m1[j] = t.m1[o + j * LPR]; v1[j] = t.v1[o + j * LPR];
    }
    for (int32_t q = fmin + 1; q <= fmax; ++q) {   // owed by some rows of the wave only
      const float ra = table[4 * q + 2], rb = table[4 * q + 3];
      if (q > fe) {
#pragma unroll
        for (int j = 0; j < EPL; ++j) {
          adam0(p0[j], m0[j], v0[j], ra, rb, s);
          adam0(p1[j], m1[j], v1[j], ra, rb, s);
        }
      }
    }
    if (fmax < target) replay_uniform<EPL, true>(p0, m0, v0, p1, m1, v1, fmax, target, table, s);
    if (valid && fe < target) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        t.p0[o + j * LPR] = p0[j]; t.m0[o + j * LPR] = m0[j]; t.v0[o + j * LPR] = v0[j];
        t.p1[o + j * LPR] = p1[j]; t.m1[o + j * LPR] = m1[j]; t.v1[o + j * LPR] = v1[j];
      }
      if (sub == 0) a.stamp[k][row] = target;
    }
  }
}

// Timing probes only (results NOT bit-identical): the replay with the square root (MODE 1), the
// reciprocal (MODE 2) or both (MODE 3) replaced by a multiply, MODE 4: v_rsq instead of sqrt,
// one row per wave as the library kernel.
template <int MODE>
__device__ __forceinline__ void adam0f(float& p, float& m, float& v, float ra, float rb, const AdamScalars& s) {
  m = __builtin_fmaf(s.b1, m, s.k1 * p);
  v = __builtin_fmaf(s.k2 * p, p, v * s.b2);
  float sq;
  if (MODE & 1) sq = v * 1.0001f;
  else if (MODE == 4) sq = v * __builtin_amdgcn_rsqf(v);
  else sq = __builtin_amdgcn_sqrtf(v);
  const float den = __builtin_fmaf(sq, ra, rb);
  const float r = (MODE & 2) ? den * 0.999f : __builtin_amdgcn_rcpf(den);
  p = __builtin_fmaf(m, r, p);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_sweep_fake(const PairArgs a, int32_t every, int32_t step_rel,
                                                    const ncf_step_clock* __restrict__ clock,
                                                    const float* __restrict__ table, AdamScalars s) {
  constexpr int D = 64;
  const int32_t target = clock->t + step_rel;
  int64_t row0[2], nrow[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t slice = (a.rows[k] + every - 1) / every;
    row0[k] = (int64_t)(target % every) * slice;
    nrow[k] = max((int64_t)0, min(slice, a.rows[k] - row0[k]));
  }
  const int64_t total = nrow[0] + nrow[1];
  const int lane = threadIdx.x & 63;
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (e >= total) return;
  const int k = e < nrow[0] ? 0 : 1;
  const int64_t row = row0[k] + (k ? e - nrow[0] : e);
  const TablePtrs& t = a.t[k];
  const int32_t from = __builtin_amdgcn_readfirstlane(a.stamp[k][row]);
  if (from >= target) return;
  const int64_t o = row * D + lane;
  float p0 = t.p0[o], m0 = t.m0[o], v0 = t.v0[o], p1 = t.p1[o], m1 = t.m1[o], v1 = t.v1[o];
  for (int32_t q = from + 1; q <= target; ++q) {
    const float ra = table[4 * q + 2], rb = table[4 * q + 3];
    adam0f<MODE>(p0, m0, v0, ra, rb, s);
    adam0f<MODE>(p1, m1, v1, ra, rb, s);
  }
  t.p0[o] = p0; t.m0[o] = m0; t.v0[o] = v0; t.p1[o] = p1; t.m1[o] = m1; t.v1[o] = v1;
  if (lane == 0) a.stamp[k][row] = target;
}

struct Tables {
  float* buf[2][6];
  int32_t* stamp[2];
  int64_t rows[2];
};

void fill_state(Tables& T, int32_t target, unsigned seed, std::vector<std::vector<float>>& host,
                std::vector<std::vector<int32_t>>& hstamp) {
  srand(seed);
  host.assign(12, {});
  hstamp.assign(2, {});
  for (int k = 0; k < 2; ++k) {
    const int64_t n = T.rows[k] * 64;
    for (int j = 0; j < 6; ++j) {
      std::vector<float>& h = host[k * 6 + j];
      h.resize(n);
      for (int64_t i = 0; i < n; ++i) {
        const float u = (float)rand() / RAND_MAX;
        h[i] = (j % 3 == 0) ? (u - 0.5f) * 0.2f : (j % 3 == 1) ? (u - 0.5f) * 1e-4f : u * 1e-7f;
      }
    }
    hstamp[k].resize(T.rows[k]);
    for (int64_t r = 0; r < T.rows[k]; ++r)
      hstamp[k][r] = (rand() % 4) ? target - 64 : target - 1 - rand() % 63;
  }
}

void upload(Tables& T, const std::vector<std::vector<float>>& host,
            const std::vector<std::vector<int32_t>>& hstamp) {
  for (int k = 0; k < 2; ++k) {
    for (int j = 0; j < 6; ++j)
      CK(hipMemcpy(T.buf[k][j], host[k * 6 + j].data(), host[k * 6 + j].size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(T.stamp[k], hstamp[k].data(), hstamp[k].size() * 4, hipMemcpyHostToDevice));
  }
}

bool same(Tables& T, const std::vector<std::vector<float>>& ref, const std::vector<std::vector<int32_t>>& rstamp) {
  for (int k = 0; k < 2; ++k) {
    for (int j = 0; j < 6; ++j) {
      std::vector<float> h(ref[k * 6 + j].size());
      CK(hipMemcpy(h.data(), T.buf[k][j], h.size() * 4, hipMemcpyDeviceToHost));
      if (memcmp(h.data(), ref[k * 6 + j].data(), h.size() * 4)) return false;
    }
    std::vector<int32_t> h(rstamp[k].size());
    CK(hipMemcpy(h.data(), T.stamp[k], h.size() * 4, hipMemcpyDeviceToHost));
    if (memcmp(h.data(), rstamp[k].data(), h.size() * 4)) return false;
  }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  const int every = 64;
  const int32_t target = 1000;   // the slice swept: target % 64
  Tables T;
  T.rows[0] = 1000000;
  T.rows[1] = 100000;
  for (int k = 0; k < 2; ++k) {
    for (int j = 0; j < 6; ++j) CK(hipMalloc(&T.buf[k][j], T.rows[k] * 64 * 4));
    CK(hipMalloc(&T.stamp[k], T.rows[k] * 4));
  }
  PairArgs a;
  memset(&a, 0, sizeof(a));
  for (int k = 0; k < 2; ++k) {
    a.t[k] = TablePtrs{T.buf[k][0], T.buf[k][1], T.buf[k][2], T.buf[k][3], T.buf[k][4], T.buf[k][5], nullptr, nullptr};
    a.stamp[k] = T.stamp[k];
    a.rows[k] = T.rows[k];
  }
  ncf_step_clock hc{target, 0, 0};
  ncf_step_clock* clock;
  CK(hipMalloc(&clock, sizeof(hc)));
  CK(hipMemcpy(clock, &hc, sizeof(hc), hipMemcpyHostToDevice));
  const int nsteps = target + 4096 + 64;
  std::vector<float> htab(4 * (nsteps + 1), 0.f);
  ncf_adam_step_scalars(1e-3, 0.9, 0.999, 1e-8, 1, nsteps, htab.data() + 4);
  float* table;
  CK(hipMalloc(&table, htab.size() * 4));
  CK(hipMemcpy(table, htab.data(), htab.size() * 4, hipMemcpyHostToDevice));
  const AdamScalars s = consts_of(0.9, 0.999, 1e-8, 1e-5);

  std::vector<std::vector<float>> h0, ref;
  std::vector<std::vector<int32_t>> s0, rs;
  fill_state(T, target, 7, h0, s0);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  // reference: the library entry point
  upload(T, h0, s0);
  ncf_table_pair pairs[2];
  memset(pairs, 0, sizeof(pairs));
  for (int k = 0; k < 2; ++k) {
    pairs[k].p0 = T.buf[k][0]; pairs[k].m0 = T.buf[k][1]; pairs[k].v0 = T.buf[k][2];
    pairs[k].p1 = T.buf[k][3]; pairs[k].m1 = T.buf[k][4]; pairs[k].v1 = T.buf[k][5];
    pairs[k].stamp = T.stamp[k];
    pairs[k].rows = T.rows[k];
  }
  if (ncf_adam_pairs_sweep_rolling(pairs, 2, 64, every, 0, clock, table, 0.9, 0.999, 1e-8, 1e-5, nullptr)) {
    fprintf(stderr, "ref: %s\n", ncf_last_error());
    return 2;
  }
  CK(hipDeviceSynchronize());
  ref.assign(12, {});
  rs.assign(2, {});
  for (int k = 0; k < 2; ++k) {
    for (int j = 0; j < 6; ++j) {
      ref[k * 6 + j].resize(T.rows[k] * 64);
      CK(hipMemcpy(ref[k * 6 + j].data(), T.buf[k][j], T.rows[k] * 64 * 4, hipMemcpyDeviceToHost));
    }
    rs[k].resize(T.rows[k]);
    CK(hipMemcpy(rs[k].data(), T.stamp[k], T.rows[k] * 4, hipMemcpyDeviceToHost));
  }

  const int64_t slice0 = (T.rows[0] + every - 1) / every, slice1 = (T.rows[1] + every - 1) / every;
  struct Var {
    const char* name;
    int id;
    int grid;
  };
  std::vector<Var> vars = {{"lib", 0, 0},
                           {"v2 flat grid", 2, 0},
                           {"v1 persistent 16 blk/CU", 1, 256 * 16},
                           {"v3 2 rows/wave", 32, 0},
                           {"v3 4 rows/wave", 34, 0},
                           {"fake0 (exact, simple loop)", 40, 0},
                           {"fake1 no sqrt", 41, 0},
                           {"fake2 no rcp", 42, 0},
                           {"fake3 no trans", 43, 0},
                           {"fake4 rsq", 44, 0}};
  auto launch = [&](const Var& v) {
    if (v.id == 0) {
      ncf_adam_pairs_sweep_rolling(pairs, 2, 64, every, 0, clock, table, 0.9, 0.999, 1e-8, 1e-5, nullptr);
    } else if (v.id == 2) {
      hipLaunchKernelGGL(k_sweep_v2<64>, dim3(grid_for((slice0 + slice1) * 64)), dim3(256), 0, 0, a, every, 0, clock, table, s);
    } else if (v.id >= 40) {
      const int g = (int)((slice0 + slice1 + 3) / 4);
      switch (v.id) {
        case 40: hipLaunchKernelGGL(k_sweep_fake<0>, dim3(g), dim3(256), 0, 0, a, every, 0, clock, table, s); break;
        case 41: hipLaunchKernelGGL(k_sweep_fake<1>, dim3(g), dim3(256), 0, 0, a, every, 0, clock, table, s); break;
        case 42: hipLaunchKernelGGL(k_sweep_fake<2>, dim3(g), dim3(256), 0, 0, a, every, 0, clock, table, s); break;
        case 43: hipLaunchKernelGGL(k_sweep_fake<3>, dim3(g), dim3(256), 0, 0, a, every, 0, clock, table, s); break;
        default: hipLaunchKernelGGL(k_sweep_fake<4>, dim3(g), dim3(256), 0, 0, a, every, 0, clock, table, s); break;
      }
    } else if (v.id == 32 || v.id == 34) {
      const int rpw = v.id == 32 ? 2 : 4;
      const int g = v.grid ? v.grid : (int)((slice0 + slice1 + 4 * rpw - 1) / (4 * rpw));
      if (rpw == 2)
        hipLaunchKernelGGL(k_sweep_v3<2>, dim3(g), dim3(256), 0, 0, a, every, 0, clock, table, s);
      else
        hipLaunchKernelGGL(k_sweep_v3<4>, dim3(g), dim3(256), 0, 0, a, every, 0, clock, table, s);
    } else {
      hipLaunchKernelGGL(k_sweep_v1<64>, dim3(v.grid), dim3(256), 0, 0, a, every, 0, clock, table, s);
    }
  };
  for (const Var& v : vars) {
    upload(T, h0, s0);
    launch(v);
    CK(hipDeviceSynchronize());
    const bool ok = same(T, ref, rs);
    float tot = 0.f;
    const int reps = 50;
    for (int r = 0; r < reps; ++r) {
      // restore the owed steps (stamps only: the replay arithmetic does not branch on values)
      for (int k = 0; k < 2; ++k)
        CK(hipMemcpy(T.stamp[k], s0[k].data(), s0[k].size() * 4, hipMemcpyHostToDevice));
      CK(hipEventRecord(e0, 0));
      launch(v);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
    }
    printf("%-28s %8.2f us  %s\n", v.name, 1e3f * tot / reps, ok ? "bit-identical" : "MISMATCH");
  }
  return 0;
}
