// Batch id deduplication: stable LSD radix sort of (id, position) pairs + segment / piece heads,
// users and items in the same launches (blockIdx.y = id kind).
//
// Reference: the EBC backward (nn.EmbeddingBag, sparse=False, src/model/architecture.py:286-287)
// sorts the batch indices (`_embedding_bag_dense_backward` -> index sort + segment reduce) before
// accumulating into a dense [rows, D] gradient.  Here the sorted segments drive the compact
// per-unique-id gradients instead (embedding_bwd.hip), and the same dedup feeds the deferred
// Adam's catch-up before the forward (deferred.py).
//
// Onesweep structure (4 launches + 1 memset for up to 2^22 rows, was 13 launches):
//   k_keys_hist   keys/positions + the digit histograms of EVERY pass (integer atomics: the
//                 totals are order-free, so deterministic);
//   k_onesweep    one launch per pass: a tile (1024 keys) ranks its keys stably in LDS (per-wave
//                 ballots), publishes its per-digit counts and finds the counts of all earlier
//                 tiles by decoupled look-back (tiles take tickets in launch order, so every
//                 predecessor is already running: no deadlock), then scatters;
//   k_segments    segment heads (id changes) and piece heads (segment heads + every sorted
//                 position multiple of PIECE), their global ranks by the same look-back, and the
//                 compact outputs: uniq ids, starts, slot maps, pieces.
// Every output is a pure function of the input ids: bitwise reproducible.
#include "segments.h"

using namespace ncf_seg;

namespace {

constexpr uint32_t ST_AGG = 1u << 30, ST_INCL = 2u << 30, ST_MASK = (1u << 30) - 1;
// up to this many tiles per kind, a tile sums all predecessors' aggregates directly (one round of
// independent loads); beyond it, the classic chained look-back (work linear in the tile count)
constexpr int kDirectTiles = 64;

__device__ __forceinline__ uint32_t ld_status(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_status64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t clamp_key(int64_t id, int64_t rows) {
  return (id < 0 || id >= rows) ? 0u : (uint32_t)id;
}

// keys (clamped ids), positions, and the digit histograms of all passes
__global__ __launch_bounds__(256) void k_keys_hist(
    const int64_t* __restrict__ ids0, int64_t rows0, const int64_t* __restrict__ ids1,
    int64_t rows1, int64_t n0, int64_t n1, int bits, int passes, uint32_t* __restrict__ k0,
    uint32_t* __restrict__ v0, uint32_t* __restrict__ k1, uint32_t* __restrict__ v1,
    uint32_t* __restrict__ ghist, uint32_t* __restrict__ num_unique, uint32_t* __restrict__ start0,
    uint32_t* __restrict__ start1, uint32_t* __restrict__ pstart0, uint32_t* __restrict__ pstart1,
    uint32_t* __restrict__ fpiece0, uint32_t* __restrict__ fpiece1) {
  __shared__ uint32_t h[MAXP][MAXR];
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  const int64_t rows = kind ? rows1 : rows0;
  const int64_t* ids = kind ? ids1 : ids0;
  uint32_t* k = kind ? k1 : k0;
  uint32_t* v = kind ? v1 : v0;
  const int R = 1 << bits;
  if (n == 0) {  // empty kind: an empty dedup (the other kernels skip it)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (num_unique) num_unique[kind] = 0;
      (kind ? start1 : start0)[0] = 0;
      (kind ? pstart1 : pstart0)[0] = 0;
      (kind ? fpiece1 : fpiece0)[0] = 0;
    }
    return;
  }
  if ((int64_t)blockIdx.x * TILE >= n) return;
  for (int i = threadIdx.x; i < passes * MAXR; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
    if (i < n) {
      const uint32_t key = clamp_key(ids[i], rows);
      k[i] = key;
      v[i] = (uint32_t)i;
      for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(key >> (p * bits)) & (R - 1)], 1u);
    }
  }
  __syncthreads();
  for (int p = 0; p < passes; ++p)
    for (int d = threadIdx.x; d < R; d += 256)
      if (h[p][d]) atomicAdd(&ghist[((int64_t)p * 2 + kind) * MAXR + d], h[p][d]);
}

// One radix pass (digit = (key >> shift) & (R-1)) with decoupled look-back over tiles.
__global__ __launch_bounds__(256) void k_onesweep(
    const uint32_t* __restrict__ kin0, const uint32_t* __restrict__ vin0,
    const uint32_t* __restrict__ kin1, const uint32_t* __restrict__ vin1, int64_t n0, int64_t n1,
    int shift, int bits, const uint32_t* __restrict__ ghist, uint32_t* __restrict__ status,
    int nbmax, uint32_t* __restrict__ tickets, uint32_t* __restrict__ kout0,
    uint32_t* __restrict__ vout0, uint32_t* __restrict__ kout1, uint32_t* __restrict__ vout1) {
  __shared__ uint32_t wcnt[4][MAXR];
  __shared__ uint32_t tcnt[MAXR];
  __shared__ uint32_t base[MAXR];
  __shared__ uint32_t csum[256];
  __shared__ uint32_t s_tile;
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  if (n == 0) return;
  const int nb = (int)((n + TILE - 1) / TILE);
  const int R = 1 << bits;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(&tickets[kind], 1u);
  for (int i = tid; i < 4 * R; i += 256) wcnt[i / R][i % R] = 0;
  __syncthreads();
  const int tile = (int)s_tile;
  if (tile >= nb) return;
  const uint32_t* kin = kind ? kin1 : kin0;
  const uint32_t* vin = kind ? vin1 : vin0;
  uint32_t* kout = kind ? kout1 : kout0;
  uint32_t* vout = kind ? vout1 : vout0;
  uint32_t* st = status + ((int64_t)kind * nbmax) * R;

  // ---- stable in-tile ranks: wave w owns keys [tile*TILE + 256w, +256) in 4 ordered steps
  const int64_t kb = (int64_t)tile * TILE + w * 256;
  uint32_t key[4], val[4], dig[4], loc[4];
  bool ok[4];
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int64_t i = kb + it * 64 + lane;
    ok[it] = i < n;
    key[it] = ok[it] ? kin[i] : 0u;
    val[it] = ok[it] ? vin[i] : 0u;
    dig[it] = (key[it] >> shift) & (uint32_t)(R - 1);
    uint64_t peers = __ballot(ok[it]);
    for (int b = 0; b < bits; ++b) {
      const uint64_t bb = __ballot((dig[it] >> b) & 1u);
      peers &= ((dig[it] >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t before = (uint32_t)__popcll(peers & lt);
    uint32_t c = 0;
    if (ok[it]) c = wcnt[w][dig[it]];
    __builtin_amdgcn_wave_barrier();
    loc[it] = c + before;
    if (ok[it] && before == 0) wcnt[w][dig[it]] = c + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // per digit: exclusive over waves (stays in wcnt), tile count -> publish aggregate
  for (int d = tid; d < R; d += 256) {
    uint32_t run = 0;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const uint32_t c = wcnt[ww][d];
      wcnt[ww][d] = run;
      run += c;
    }
    tcnt[d] = run;
    st_status(&st[(int64_t)tile * R + d], (tile == 0 ? ST_INCL : ST_AGG) | run);
  }
  // global digit starts: exclusive scan of this pass's histogram (chunk per thread + LDS scan)
  const uint32_t* gh = ghist + (int64_t)kind * MAXR;
  const int per = (R + 255) / 256;
  uint32_t mine = 0;
  for (int j = 0; j < per; ++j) {
    const int d = tid * per + j;
    if (d < R) mine += gh[d];
  }
  csum[tid] = mine;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const uint32_t x = tid >= off ? csum[tid - off] : 0u;
    __syncthreads();
    csum[tid] += x;
    __syncthreads();
  }
  {
    uint32_t run = csum[tid] - mine;
    for (int j = 0; j < per; ++j) {
      const int d = tid * per + j;
      if (d < R) {
        base[d] = run;
        run += gh[d];
      }
    }
  }
  __syncthreads();
  if (nb <= kDirectTiles) {
    // few tiles: sum the aggregates of ALL earlier tiles directly (independent loads, 2 digits
    // per 64-bit load, 8 tiles per batch) instead of walking an inclusive-prefix chain
    const uint64_t* st64 = reinterpret_cast<const uint64_t*>(st);
    for (int d0 = 2 * tid; d0 < R; d0 += 512) {
      uint32_t e0 = 0, e1 = 0;
      for (int tb = 0; tb < tile; tb += 8) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = tb + j < tile ? ld_status64(&st64[((int64_t)(tb + j) * R + d0) / 2])
                               : ((uint64_t)ST_AGG << 32 | ST_AGG);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          while (((uint32_t)v[j] & ~ST_MASK) == 0 || ((uint32_t)(v[j] >> 32) & ~ST_MASK) == 0) {
            __builtin_amdgcn_s_sleep(1);
            v[j] = ld_status64(&st64[((int64_t)(tb + j) * R + d0) / 2]);
          }
          e0 += (uint32_t)v[j] & ST_MASK;
          e1 += (uint32_t)(v[j] >> 32) & ST_MASK;
        }
      }
      base[d0] += e0;
      base[d0 + 1] += e1;
    }
  } else {
    // decoupled look-back: counts of this digit in all earlier tiles
    for (int d = tid; d < R; d += 256) {
      uint32_t excl = 0;
      if (tile > 0) {
        int t = tile - 1;
        while (true) {
          const uint32_t s = ld_status(&st[(int64_t)t * R + d]);
          if ((s & ~ST_MASK) == 0) {
            __builtin_amdgcn_s_sleep(1);
            continue;
          }
          excl += s & ST_MASK;
          if (s & ST_INCL) break;
          --t;
        }
        st_status(&st[(int64_t)tile * R + d], ST_INCL | (excl + tcnt[d]));
      }
      base[d] += excl;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    if (!ok[it]) continue;
    const uint32_t pos = base[dig[it]] + wcnt[w][dig[it]] + loc[it];
    kout[pos] = key[it];
    vout[pos] = val[it];
  }
}

// Segment heads (sorted key changes) and piece heads (segment heads + positions multiple of
// PIECE), ranked globally by look-back on packed (segments, pieces) tile counts.
__global__ __launch_bounds__(256) void k_segments(
    const uint32_t* __restrict__ sk0, const uint32_t* __restrict__ sk1, int64_t n0, int64_t n1,
    int nbmax, uint64_t* __restrict__ sstatus, uint32_t* __restrict__ tickets,
    uint32_t* __restrict__ segoff, uint32_t* __restrict__ start0, uint32_t* __restrict__ start1,
    uint32_t* __restrict__ pstart0, uint32_t* __restrict__ pstart1, uint32_t* __restrict__ pseg0,
    uint32_t* __restrict__ pseg1, uint32_t* __restrict__ fpiece0, uint32_t* __restrict__ fpiece1,
    int64_t* __restrict__ uniq0, int64_t* __restrict__ uniq1, int32_t* __restrict__ slot0,
    int32_t* __restrict__ slot1, uint32_t* __restrict__ totals, uint32_t* __restrict__ num_unique) {
  constexpr uint64_t F_AGG = 1ull << 62, F_INCL = 2ull << 62, M31 = (1ull << 31) - 1;
  __shared__ uint32_t ws_s[16], ws_p[16];
  __shared__ uint32_t s_tile, s_es, s_ep;
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  if (n == 0) return;
  const int nb = (int)((n + TILE - 1) / TILE);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(&tickets[kind], 1u);
  __syncthreads();
  const int tile = (int)s_tile;
  if (tile >= nb) return;
  const uint32_t* sk = kind ? sk1 : sk0;
  uint64_t* st = sstatus + (int64_t)kind * nbmax;
  const uint64_t le = (lane == 63) ? ~0ull : ((1ull << (lane + 1)) - 1);  // inclusive
  bool sh[4], ph[4];
  uint32_t sr[4], pr[4], key[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)tile * TILE + r * 256 + tid;
    key[r] = i < n ? sk[i] : 0u;
    sh[r] = i < n && (i == 0 || key[r] != sk[i - 1]);
    ph[r] = i < n && (sh[r] || (i % PIECE) == 0);
    const uint64_t ms = __ballot(sh[r]), mp = __ballot(ph[r]);
    sr[r] = (uint32_t)__popcll(ms & le);
    pr[r] = (uint32_t)__popcll(mp & le);
    if (lane == 0) {
      ws_s[r * 4 + w] = (uint32_t)__popcll(ms);
      ws_p[r * 4 + w] = (uint32_t)__popcll(mp);
    }
  }
  __syncthreads();
  if (w == 0) {
    uint64_t S = 0, Pc = 0;
    for (int q = 0; q < 16; ++q) { S += ws_s[q]; Pc += ws_p[q]; }
    uint64_t es = 0, ep = 0;
    if (nb <= kDirectTiles) {
      // all predecessors at once: lane j reads tile j's aggregate
      if (lane == 0) st_status64(&st[tile], F_AGG | (S << 31) | Pc);
      uint64_t v = 0;
      if (lane < tile) {
        do {
          v = ld_status64(&st[lane]);
          if ((v >> 62) == 0) __builtin_amdgcn_s_sleep(1);
        } while ((v >> 62) == 0);
      }
      uint32_t a = (uint32_t)((v >> 31) & M31), b = (uint32_t)(v & M31);  // totals < 2^30
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
      }
      es = a;
      ep = b;
    } else if (lane == 0) {
      if (tile == 0) {
        st_status64(&st[0], F_INCL | (S << 31) | Pc);
      } else {
        st_status64(&st[tile], F_AGG | (S << 31) | Pc);
        int t = tile - 1;
        while (true) {
          const uint64_t s = ld_status64(&st[t]);
          if ((s >> 62) == 0) {
            __builtin_amdgcn_s_sleep(1);
            continue;
          }
          es += (s >> 31) & M31;
          ep += s & M31;
          if (s & F_INCL) break;
          --t;
        }
        st_status64(&st[tile], F_INCL | ((es + S) << 31) | (ep + Pc));
      }
    }
    if (lane == 0) {
      s_es = (uint32_t)es;
      s_ep = (uint32_t)ep;
      segoff[(int64_t)kind * nbmax + tile] = (uint32_t)es;
      if (tile == nb - 1) {
        const uint32_t U = (uint32_t)(es + S), Pn = (uint32_t)(ep + Pc);
        totals[kind] = U;
        totals[2 + kind] = Pn;
        if (num_unique) num_unique[kind] = U;
        (kind ? start1 : start0)[U] = (uint32_t)n;
        (kind ? pstart1 : pstart0)[Pn] = (uint32_t)n;
        (kind ? fpiece1 : fpiece0)[U] = Pn;
      }
    }
  }
  __syncthreads();
  uint32_t* start = kind ? start1 : start0;
  uint32_t* pstart = kind ? pstart1 : pstart0;
  uint32_t* pseg = kind ? pseg1 : pseg0;
  uint32_t* fpiece = kind ? fpiece1 : fpiece0;
  int64_t* uniq = kind ? uniq1 : uniq0;
  int32_t* slot = kind ? slot1 : slot0;
  uint32_t bs = s_es, bp = s_ep;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint32_t pre_s = 0, pre_p = 0;
    for (int q = 0; q < r * 4 + w; ++q) { pre_s += ws_s[q]; pre_p += ws_p[q]; }
    const int64_t i = (int64_t)tile * TILE + r * 256 + tid;
    if (i >= n) continue;
    const uint32_t c = bs + pre_s + sr[r] - 1;  // segment of position i
    if (sh[r]) {
      start[c] = (uint32_t)i;
      uniq[c] = (int64_t)key[r];
      if (slot) slot[key[r]] = (int32_t)c;
    }
    if (ph[r]) {
      const uint32_t p = bp + pre_p + pr[r] - 1;
      pstart[p] = (uint32_t)i;
      pseg[p] = c | (sh[r] ? FIRST_PIECE : 0u);
      if (sh[r]) fpiece[c] = p;
    }
  }
}

// ---- small batches (every kind <= kSmallMax ids): the whole dedup in ONE launch, one workgroup
// per kind.  The (key, position) pairs sort as 64-bit words (key << 32 | position: the stable
// order of the radix sort, positions breaking ties) by a bitonic network in LDS, then the segment
// and piece heads are ranked by a workgroup scan.  Every output the multi-launch path leaves in
// the workspace (sorted pairs in the buffers its pass count ends in, segments, pieces, segment
// offsets per sort tile, totals, uniq ids, slot maps, counts) is written with the same values.
// The reference call pattern's batch (config.yaml:65: 256 groups of 5 = 1,280 ids) sorted in 5
// dependent launches (a memset, keys + histograms, two radix passes, segments) took ~37 us.
constexpr int kSmallMax = 2048;
__global__ __launch_bounds__(1024) void k_dedup_small(
    const int64_t* __restrict__ ids0, int64_t rows0, const int64_t* __restrict__ ids1,
    int64_t rows1, int64_t n0, int64_t n1, int nbmax, uint32_t* __restrict__ ko0,
    uint32_t* __restrict__ vo0, uint32_t* __restrict__ ko1, uint32_t* __restrict__ vo1,
    uint32_t* __restrict__ segoff, uint32_t* __restrict__ start0, uint32_t* __restrict__ start1,
    uint32_t* __restrict__ pstart0, uint32_t* __restrict__ pstart1, uint32_t* __restrict__ pseg0,
    uint32_t* __restrict__ pseg1, uint32_t* __restrict__ fpiece0, uint32_t* __restrict__ fpiece1,
    int64_t* __restrict__ uniq0, int64_t* __restrict__ uniq1, int32_t* __restrict__ slot0,
    int32_t* __restrict__ slot1, uint32_t* __restrict__ totals, uint32_t* __restrict__ num_unique) {
  __shared__ uint64_t s[kSmallMax];
  __shared__ uint32_t wsum_s[16], wsum_p[16];
  const int kind = blockIdx.y;
  const int n = (int)(kind ? n1 : n0);
  const int64_t rows = kind ? rows1 : rows0;
  const int64_t* ids = kind ? ids1 : ids0;
  uint32_t* ko = kind ? ko1 : ko0;
  uint32_t* vo = kind ? vo1 : vo0;
  uint32_t* start = kind ? start1 : start0;
  uint32_t* pstart = kind ? pstart1 : pstart0;
  uint32_t* pseg = kind ? pseg1 : pseg0;
  uint32_t* fpiece = kind ? fpiece1 : fpiece0;
  int64_t* uniq = kind ? uniq1 : uniq0;
  int32_t* slot = kind ? slot1 : slot0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (n == 0) {
    if (tid == 0) {
      if (num_unique) num_unique[kind] = 0;
      totals[kind] = 0;
      totals[2 + kind] = 0;
      start[0] = 0;
      pstart[0] = 0;
      fpiece[0] = 0;
    }
    return;
  }
  int N2 = 2;
  while (N2 < n) N2 <<= 1;
  for (int i = tid; i < N2; i += 1024)
    s[i] = i < n ? ((uint64_t)clamp_key(ids[i], rows) << 32 | (uint32_t)i) : ~0ull;
  __syncthreads();
  // bitonic sort, ascending: N2 / 2 compare-exchanges per stage, one per thread (N2 <= 2048)
  for (int k = 2; k <= N2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = tid; t < (N2 >> 1); t += 1024) {
        const int i = 2 * j * (t / j) + (t % j), l = i + j;
        const uint64_t a = s[i], b = s[l];
        const bool up = (i & k) == 0;
        if ((a > b) == up) { s[i] = b; s[l] = a; }
      }
      __syncthreads();
    }
  }
  // heads: thread tid holds sorted positions 2 tid and 2 tid + 1
  uint32_t key[2], cs[2], cp[2];
  bool sh[2], ph[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int i = 2 * tid + e;
    key[e] = i < n ? (uint32_t)(s[i] >> 32) : 0u;
    sh[e] = i < n && (i == 0 || key[e] != (uint32_t)(s[i - 1] >> 32));
    ph[e] = i < n && (sh[e] || (i % PIECE) == 0);
  }
  // inclusive ranks: within the thread, the wave (ballot counts), then the earlier waves
  const uint32_t ts = (uint32_t)sh[0] + (uint32_t)sh[1], tp = (uint32_t)ph[0] + (uint32_t)ph[1];
  uint32_t is = ts, ip = tp;   // inclusive wave scans of the per-thread counts
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t xs = __shfl_up(is, o, 64), xp = __shfl_up(ip, o, 64);
    if (lane >= o) { is += xs; ip += xp; }
  }
  if (lane == 63) { wsum_s[w] = is; wsum_p[w] = ip; }
  __syncthreads();
  uint32_t bs = 0, bp = 0, U = 0, Pn = 0;
  for (int q = 0; q < 16; ++q) {
    if (q < w) { bs += wsum_s[q]; bp += wsum_p[q]; }
    U += wsum_s[q];
    Pn += wsum_p[q];
  }
  cs[0] = bs + is - ts + (uint32_t)sh[0];   // inclusive segment count at position 2 tid
  cs[1] = cs[0] + (uint32_t)sh[1];
  cp[0] = bp + ip - tp + (uint32_t)ph[0];
  cp[1] = cp[0] + (uint32_t)ph[1];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int i = 2 * tid + e;
    if (i >= n) continue;
    ko[i] = key[e];
    vo[i] = (uint32_t)s[i];
    const uint32_t c = cs[e] - 1;   // segment of position i
    if (sh[e]) {
      start[c] = (uint32_t)i;
      uniq[c] = (int64_t)key[e];
      if (slot) slot[key[e]] = (int32_t)c;
    }
    if (ph[e]) {
      const uint32_t p = cp[e] - 1;
      pstart[p] = (uint32_t)i;
      pseg[p] = c | (sh[e] ? FIRST_PIECE : 0u);
      if (sh[e]) fpiece[c] = p;
    }
    // segments starting before sort tile i / TILE (the multi-launch path's look-back offsets)
    if (i % TILE == 0) segoff[(int64_t)kind * nbmax + i / TILE] = cs[e] - (uint32_t)sh[e];
  }
  if (tid == 0) {
    totals[kind] = U;
    totals[2 + kind] = Pn;
    if (num_unique) num_unique[kind] = U;
    start[U] = (uint32_t)n;
    pstart[Pn] = (uint32_t)n;
    fpiece[U] = Pn;
  }
}

// the largest per-kind id count the one-launch form takes (ncf_dedup_set_small_max: A/B, tests)
static int64_t g_small_max = kSmallMax;

// inverse map of a dedup: inv[position] = compact index of its id
__global__ __launch_bounds__(256) void k_seg_inverse(const uint32_t* __restrict__ sk0,
                                                     const uint32_t* __restrict__ sk1,
                                                     const uint32_t* __restrict__ sv0,
                                                     const uint32_t* __restrict__ sv1, int64_t n0,
                                                     int64_t n1, int nb,
                                                     const uint32_t* __restrict__ off,
                                                     int64_t* __restrict__ inv0,
                                                     int64_t* __restrict__ inv1) {
  __shared__ uint32_t wsum[16];
  const int kind = blockIdx.y;
  const int64_t n = kind ? n1 : n0;
  const uint32_t* sk = kind ? sk1 : sk0;
  const uint32_t* sv = kind ? sv1 : sv0;
  int64_t* inv = kind ? inv1 : inv0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  bool head[4];
  uint32_t rank[4];
  const uint64_t le = (lane == 63) ? ~0ull : ((1ull << (lane + 1)) - 1);  // inclusive
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
    head[r] = i < n && (i == 0 || sk[i] != sk[i - 1]);
    const uint64_t m = __ballot(head[r]);
    rank[r] = (uint32_t)__popcll(m & le);
    if (lane == 0) wsum[r * 4 + w] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  const uint32_t base = off[(int64_t)kind * nb + blockIdx.x];
  for (int r = 0; r < 4; ++r) {
    const int64_t i = (int64_t)blockIdx.x * TILE + r * 256 + threadIdx.x;
    if (i >= n) continue;
    uint32_t pre = 0;
    for (int q = 0; q < r * 4 + w; ++q) pre += wsum[q];
    inv[sv[i]] = (int64_t)(base + pre + rank[r]) - 1;
  }
}

}  // namespace

// Stable radix sort of (id, position) for two id lists (kind 0 / kind 1, lengths n0 / n1) +
// segment and piece heads: uniq ids per kind, num_unique[kind], optional slot maps.  Sorted
// positions, segments and pieces stay in `workspace` (sized for max(n0, n1)).
extern "C" int ncf_dedup_ids2(const int64_t* ids0, int64_t n0, int64_t rows0, const int64_t* ids1,
                              int64_t n1, int64_t rows1, int64_t dim, int64_t* uniq0,
                              int64_t* uniq1, int32_t* slot0, int32_t* slot1,
                              uint32_t* num_unique, void* workspace, int64_t workspace_bytes,
                              void* stream) {
  const int64_t n = n0 > n1 ? n0 : n1;
  NCF_CHECK_ARG(n0 >= 0 && n1 >= 0 && n < (1ll << 30), "ncf_dedup_ids: bad n");
  NCF_CHECK_ARG(rows0 >= 1 && rows1 >= 1 && rows0 <= (1ll << 32) && rows1 <= (1ll << 32),
                "ncf_dedup_ids: rows must be in [1, 2^32]");
  if (workspace_bytes < ws_bytes(n, dim)) {
    ncf_set_error("ncf_dedup_ids: workspace %lld < %lld bytes", (long long)workspace_bytes,
                  (long long)ws_bytes(n, dim));
    return NCF_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  WS w = carve(workspace, n, dim);
  const int passes = sort_passes(rows0, rows1), bits = digit_bits(rows0, rows1);
  if (n == 0) {
    if (num_unique) (void)hipMemsetAsync(num_unique, 0, 2 * sizeof(uint32_t), st);
    (void)hipMemsetAsync(w.totals, 0, 4 * sizeof(uint32_t), st);
    return NCF_OK;
  }
  if (n <= g_small_max) {
    uint32_t *k0, *v0, *k1, *v1;
    sorted_bufs(w, passes, &k0, &v0, &k1, &v1);
    hipLaunchKernelGGL(k_dedup_small, dim3(1, 2), dim3(1024), 0, st, ids0, rows0, ids1, rows1, n0,
                       n1, w.nb, k0, v0, k1, v1, w.segoff, w.start0, w.start1, w.pstart0,
                       w.pstart1, w.pseg0, w.pseg1, w.fpiece0, w.fpiece1, uniq0, uniq1, slot0,
                       slot1, w.totals, num_unique);
    NCF_CHECK_LAUNCH("ncf_dedup_ids(small)");
    return NCF_OK;
  }
  (void)hipMemsetAsync(workspace, 0, (size_t)w.zero_bytes(workspace, passes, bits), st);
  hipLaunchKernelGGL(k_keys_hist, dim3(w.nb, 2), dim3(256), 0, st, ids0, rows0, ids1, rows1, n0,
                     n1, bits, passes, w.ka0, w.va0, w.ka1, w.va1, w.ghist, num_unique, w.start0,
                     w.start1, w.pstart0, w.pstart1, w.fpiece0, w.fpiece1);
  NCF_CHECK_LAUNCH("ncf_dedup_ids(keys)");
  uint32_t *ki0 = w.ka0, *vi0 = w.va0, *ki1 = w.ka1, *vi1 = w.va1;
  uint32_t *ko0 = w.kb0, *vo0 = w.vb0, *ko1 = w.kb1, *vo1 = w.vb1;
  const int64_t R = 1ll << bits;
  for (int p = 0; p < passes; ++p) {
    hipLaunchKernelGGL(k_onesweep, dim3(w.nb, 2), dim3(256), 0, st, ki0, vi0, ki1, vi1, n0, n1,
                       p * bits, bits, w.ghist + (int64_t)p * 2 * MAXR,
                       w.status + (int64_t)p * 2 * w.nb * R, w.nb, w.tickets + 2 * p, ko0, vo0,
                       ko1, vo1);
    NCF_CHECK_LAUNCH("ncf_dedup_ids(sort)");
    uint32_t* t;
    t = ki0; ki0 = ko0; ko0 = t;
    t = vi0; vi0 = vo0; vo0 = t;
    t = ki1; ki1 = ko1; ko1 = t;
    t = vi1; vi1 = vo1; vo1 = t;
  }
  hipLaunchKernelGGL(k_segments, dim3(w.nb, 2), dim3(256), 0, st, ki0, ki1, n0, n1, w.nb,
                     w.sstatus, w.tickets + 2 * MAXP, w.segoff, w.start0, w.start1, w.pstart0,
                     w.pstart1, w.pseg0, w.pseg1, w.fpiece0, w.fpiece1, uniq0, uniq1,
                     slot0, slot1, w.totals, num_unique);
  NCF_CHECK_LAUNCH("ncf_dedup_ids(segments)");
  return NCF_OK;
}

extern "C" int ncf_dedup_ids(const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                             int64_t dim, int64_t num_users, int64_t num_items,
                             int64_t* uniq_users, int64_t* uniq_items, int32_t* slot_users,
                             int32_t* slot_items, uint32_t* num_unique, void* workspace,
                             int64_t workspace_bytes, void* stream) {
  return ncf_dedup_ids2(user_ids, n, num_users, item_ids, n, num_items, dim, uniq_users,
                        uniq_items, slot_users, slot_items, num_unique, workspace,
                        workspace_bytes, stream);
}

extern "C" int64_t ncf_embedding_bwd_workspace(int64_t n, int64_t dim) { return ws_bytes(n, dim); }

extern "C" int64_t ncf_dedup_set_small_max(int64_t n) {
  const int64_t prev = g_small_max;
  if (n >= 0) g_small_max = n < kSmallMax ? n : kSmallMax;
  return prev;
}

// inv[position] = compact index, for the dedup held in `workspace` (ncf_dedup_ids2, same args)
extern "C" int ncf_dedup_inverse(int64_t n0, int64_t n1, int64_t rows0, int64_t rows1, int64_t dim,
                                 int64_t* inv0, int64_t* inv1, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  const int64_t n = n0 > n1 ? n0 : n1;
  if (workspace_bytes < ws_bytes(n, dim)) {
    ncf_set_error("ncf_dedup_inverse: workspace too small");
    return NCF_ERR_WORKSPACE;
  }
  if (n == 0) return NCF_OK;
  WS w = carve(workspace, n, dim);
  uint32_t *k0, *v0, *k1, *v1;
  sorted_bufs(w, sort_passes(rows0, rows1), &k0, &v0, &k1, &v1);
  hipLaunchKernelGGL(k_seg_inverse, dim3(w.nb, 2), dim3(256), 0, (hipStream_t)stream, k0, k1, v0,
                     v1, n0, n1, w.nb, w.segoff, inv0, inv1);
  NCF_CHECK_LAUNCH("ncf_dedup_inverse");
  return NCF_OK;
}
