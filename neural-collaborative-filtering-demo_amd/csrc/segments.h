// Internal: workspace layout shared by the id dedup (dedup.hip), the embedding backward
// (embedding_bwd.hip) and the row-sharding pack/unpack kernels (shard.hip).
//
// A dedup of two id lists (kind 0 = users, kind 1 = items; lengths n0, n1 <= n) leaves in the
// workspace, per kind:
//   sorted (key, position) pairs      — stable LSD radix sort, 2 passes for <= 2^22 rows;
//   segments c = 0..U-1               — start[c] (sorted position), uniq[c] (id), U = totals[kind];
//   pieces p = 0..Pn-1                — a segment split at every sorted position multiple of
//                                       PIECE: pstart[p], pseg[p] = its segment | FIRST_PIECE
//                                       for a segment's first piece, first piece of segment
//                                       c = fpiece[c], Pn = totals[2 + kind];
//   segoff[kind][tile]                — segments starting before sort tile `tile`;
#pragma once
#include "ncf_common.h"

namespace ncf_seg {

constexpr int TILE = 1024;        // keys per sort tile (256 threads x 4)
#ifndef NCF_PIECE
#define NCF_PIECE 16
#endif
constexpr int PIECE = NCF_PIECE;  // max occurrences one lane group reduces in the embedding backward
#ifndef NCF_RADIX_BITS
#define NCF_RADIX_BITS 11
#endif
constexpr int MAX_BITS = NCF_RADIX_BITS;   // radix digit bits (at most)
constexpr int MAXR = 1 << MAX_BITS;
constexpr int MAXP = (32 + MAX_BITS - 1) / MAX_BITS;   // passes for 32-bit keys
constexpr uint32_t FIRST_PIECE = 1u << 31;

struct WS {
  // zeroed by every dedup (one memset over [tickets, status + used part)): tickets, digit
  // histograms, segment look-back status, totals, radix look-back status
  uint32_t* tickets;   // [MAXP + 1][2]
  uint32_t* ghist;     // [MAXP][2][MAXR]
  uint64_t* sstatus;   // [2][nb]
  uint32_t* totals;    // [4]: U0, U1, pieces0, pieces1
  uint32_t* status;    // [passes][2][nb][R]  (R = 2^digit_bits)
  // sort buffers (ping-pong) and the 8-bit sort of the sharding path
  uint32_t *ka0, *va0, *ka1, *va1, *kb0, *vb0, *kb1, *vb1;
  uint32_t* hist;      // [2][256][nb]
  // segments / pieces
  uint32_t* segoff;    // [2][nb]
  uint32_t *start0, *start1, *pstart0, *pstart1, *pseg0, *pseg1, *fpiece0, *fpiece1;
  float *xp0, *xp1;    // [extras][2D] LayerNorm-backward rows of the non-first pieces
  float* part;         // [2 * nbr + 1][4D] dgamma/dbeta partials
  float* red_scratch;
  int nb, nbr;
  // bytes from the workspace base that a dedup with `passes` passes of 2^bits digits zeroes
  int64_t zero_bytes(void* base, int passes, int bits) const {
    return (int64_t)((char*)status - (char*)base) + 4ll * passes * 2 * nb * (1ll << bits);
  }
};

static inline int nb_of(int64_t n) { return n == 0 ? 1 : ncf_cdiv(n, TILE); }
static inline int64_t pieces_max(int64_t n) { return n + n / PIECE + 2; }
static inline int64_t extras_max(int64_t n) { return n / PIECE + 2; }
// piece-reduce blocks: NCF_PIECE_WAVES waves, each reducing 64 / (D/4) pieces at a time (one per
// group of D/4 lanes).  4-wave blocks: the fused-apply reduce holds 164 VGPRs (3 waves per SIMD),
// so 8-wave blocks left one block (8 waves) per CU and 4-wave blocks fit three (12 waves); capped
// at 768 blocks (three per CU, grid-stride beyond) so the dgamma/dbeta partial rows stay as few as
// with 8-wave blocks.  C2, interleaved A/B (r06m, r06n): the reduce + fused apply 42.1-42.9 ->
// 36.7-37.5 us, the batch's reductions +0.7 us.
#ifndef NCF_PIECE_WAVES
#define NCF_PIECE_WAVES 4
#endif
static inline int nbr_of(int64_t n, int64_t D) {
  const int64_t per = (int64_t)NCF_PIECE_WAVES * (D >= 256 ? 1 : 256 / D);
  int64_t b = (pieces_max(n) + per - 1) / per;
  if (b < 1) b = 1;
#ifndef NCF_PIECE_BLOCKS_MAX
#define NCF_PIECE_BLOCKS_MAX 768
#endif
  if (b > NCF_PIECE_BLOCKS_MAX) b = NCF_PIECE_BLOCKS_MAX;
  return (int)b;
}

static inline int64_t round256(int64_t b) { return (b + 255) / 256 * 256; }

static inline int64_t ws_bytes(int64_t n, int64_t D) {
  const int64_t nb = nb_of(n), nbr = nbr_of(n, D);
  int64_t b = 0;
  b += round256(4 * 2 * (MAXP + 1));
  b += round256(4 * (int64_t)MAXP * 2 * MAXR);
  b += round256(8 * 2 * nb);
  b += round256(4 * 4);
  b += round256(4 * (int64_t)MAXP * 2 * nb * MAXR);
  b += 8 * round256(4 * (n + 64));
  b += round256(4 * 2 * 256 * nb);
  b += round256(4 * 2 * nb);
  b += 2 * round256(4 * (n + 2));            // start
  b += 4 * round256(4 * pieces_max(n));      // pstart, pseg
  b += 2 * round256(4 * (n + 2));            // fpiece
  b += 2 * round256(4 * extras_max(n) * 2 * D);
  b += round256(4 * (2 * nbr + 1) * 4 * D);
  b += round256(4 * ncf_reduce_scratch(2 * nbr, 4 * D) + 4);
  return b + 1024;
}

static inline WS carve(void* base, int64_t n, int64_t D) {
  WS w;
  w.nb = nb_of(n);
  w.nbr = nbr_of(n, D);
  char* p = (char*)base;
  auto take = [&](int64_t bytes) {
    char* r = p;
    p += round256(bytes);
    return r;
  };
  w.tickets = (uint32_t*)take(4 * 2 * (MAXP + 1));
  w.ghist = (uint32_t*)take(4 * (int64_t)MAXP * 2 * MAXR);
  w.sstatus = (uint64_t*)take(8 * 2 * (int64_t)w.nb);
  w.totals = (uint32_t*)take(4 * 4);
  w.status = (uint32_t*)take(4 * (int64_t)MAXP * 2 * w.nb * MAXR);
  const int64_t kb = 4 * (n + 64);
  w.ka0 = (uint32_t*)take(kb); w.va0 = (uint32_t*)take(kb);
  w.ka1 = (uint32_t*)take(kb); w.va1 = (uint32_t*)take(kb);
  w.kb0 = (uint32_t*)take(kb); w.vb0 = (uint32_t*)take(kb);
  w.kb1 = (uint32_t*)take(kb); w.vb1 = (uint32_t*)take(kb);
  w.hist = (uint32_t*)take(4 * 2 * 256 * (int64_t)w.nb);
  w.segoff = (uint32_t*)take(4 * 2 * (int64_t)w.nb);
  w.start0 = (uint32_t*)take(4 * (n + 2));
  w.start1 = (uint32_t*)take(4 * (n + 2));
  w.pstart0 = (uint32_t*)take(4 * pieces_max(n));
  w.pstart1 = (uint32_t*)take(4 * pieces_max(n));
  w.pseg0 = (uint32_t*)take(4 * pieces_max(n));
  w.pseg1 = (uint32_t*)take(4 * pieces_max(n));
  w.fpiece0 = (uint32_t*)take(4 * (n + 2));
  w.fpiece1 = (uint32_t*)take(4 * (n + 2));
  w.xp0 = (float*)take(4 * extras_max(n) * 2 * D);
  w.xp1 = (float*)take(4 * extras_max(n) * 2 * D);
  w.part = (float*)take(4 * (2 * (int64_t)w.nbr + 1) * 4 * D);
  w.red_scratch = (float*)take(4 * ncf_reduce_scratch(2 * w.nbr, 4 * D) + 4);
  return w;
}

static inline int bits_for(int64_t rows) {
  int b = 1;
  while (b < 32 && (1ll << b) < rows) ++b;
  return b;
}

// radix passes and digit width for keys < max(rows0, rows1)
static inline int sort_passes(int64_t rows0, int64_t rows1) {
  const int b = bits_for(rows0 > rows1 ? rows0 : rows1);
  return (b + MAX_BITS - 1) / MAX_BITS;
}
static inline int digit_bits(int64_t rows0, int64_t rows1) {
  const int b = bits_for(rows0 > rows1 ? rows0 : rows1);
  const int p = sort_passes(rows0, rows1);
  return (b + p - 1) / p;
}

// sorted (keys, positions) after `passes` ping-pong passes
static inline void sorted_bufs(const WS& w, int passes, uint32_t** k0, uint32_t** v0,
                               uint32_t** k1, uint32_t** v1) {
  const bool odd = passes & 1;
  *k0 = odd ? w.kb0 : w.ka0;
  *v0 = odd ? w.vb0 : w.va0;
  *k1 = odd ? w.kb1 : w.ka1;
  *v1 = odd ? w.vb1 : w.va1;
}

}  // namespace ncf_seg
