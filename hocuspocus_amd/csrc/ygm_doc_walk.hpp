// ygm_doc_walk.hpp -- encodeStateVectorFromUpdate / diffUpdate fast path (the
// reconnect-sync shape): ONE LANE PER DOCUMENT, 64 documents of a wave walked side by side, each
// lane streaming its document through a private ring in LDS.
//
// Why lane-per-document: a V1 update is a chain -- every struct's start is the previous struct's
// end, and a client block's extent is known only by counting its structs.  Splitting one 1-8 KB
// document over a wave needs a resolution pass per client block (the speculative walks cross block
// headers blind), which costs more wave instructions than the walk itself; 64 documents give 64
// independent chains for free.  What made the round-1 walker slow was not the mapping but ~1000
// VALU per struct (a 64-byte register window shifted by moves, full byte views, per-byte stores)
// and loads that every iteration waited on.  Here:
//   * staging: per round each lane loads its next one or two 64-byte chunks (16-byte loads) into
//     registers; they are written to the lane's ring (4 chunk slots) at the next round start, so a
//     load has a whole round (DW_R iterations) to land.  No other vector-memory instruction runs
//     inside the parse iterations: output bytes, copy runs and finished documents are written at
//     the round start, after the staged loads have been waited on and before new ones are issued
//     (vmcnt is in order on gfx950: a store issued mid-round would be waited on by the next load
//     use).
//   * struct boundaries: when a chunk lands its terminator mask (bit = byte with the top bit clear,
//     i.e. the end of a varuint) is built by v_dot4 from its 16 dwords and kept in LDS; a struct's
//     varuint ends are the k-th set bits of the 64-bit mask window at its start (popcount-select:
//     clear-lowest + ctz), its string bytes are checked ASCII against the same mask, and only the
//     content-length bytes are read.  Non-minimal varuints (a top-bit byte followed by 0x00) and
//     varuints of >= 6 bytes are found per chunk from the same masks.
//   * diff output: the block header (and, when the state vector cuts a struct, its re-encoded
//     prefix) is written at the round start; the verbatim rest of the client block streams from
//     the ring to the output in 16-byte pieces as the walk passes it (no second read of the input).
//
// Rules: R-SV (yjs Y@37728) and R-D (App. B.2, Y@40711), restated from sv_doc /
// DiffGen (ygm_seqdoc.hpp), which stay the exact reference for what this kernel defers: content other
// than String (ASCII) / Deleted / Type / Binary, items with parent info other than 0 / 1, info bit
// 0x20 beside an origin, GC info bytes other than 0, values >= 2^32, blocks not strictly
// client-descending or empty, delete sets not strictly client-descending or with empty clients,
// state vectors of > 16 entries or with trailing bytes, outputs over the slot, documents >= 1 GB.
#pragma once
#include "ygm_merge_lean.hpp"

namespace ygm {

#ifndef YGM_DW_S
#define YGM_DW_S 4
#endif
constexpr int DW_S = YGM_DW_S;    // 64-byte chunk slots per lane ring (a power of two)
constexpr int DW_P = DW_S * 4;    // 16-byte pieces per ring
#ifndef YGM_DW_R
#define YGM_DW_R 4
#endif
#ifndef YGM_DW_STG
#define YGM_DW_STG 3
#endif
#ifndef YGM_DW_U
#define YGM_DW_U 3
#endif
constexpr int DW_R = YGM_DW_R;    // parse iterations per round
constexpr int DW_U = YGM_DW_U;    // Items the fast decoder takes per iteration (from one 64-byte mask window): SV
constexpr int DW_U1 = DW_U + 1;   // ... diff (its per-iteration and per-round overhead is larger: 4 measured 2 % faster)
constexpr uint32_t DW_STG = YGM_DW_STG;   // chunks staged per round (<= 4: 64 staging registers)
#ifndef YGM_DW_AHEAD
#define YGM_DW_AHEAD 2
#endif
constexpr uint32_t DW_AHEAD = YGM_DW_AHEAD;  // chunks staged past the ring's free slots (committed if the round freed theirs)
constexpr int DW_BATCH = 256;     // documents sorted (largest first) per batch of a wave's range
constexpr int DW_SVN = 16;        // state-vector entries per lane (diff)
constexpr uint32_t DW_OPEN = 0xFFFFFFFFu;

#ifndef YGM_DW_LM
#define YGM_DW_LM 1
#endif
// The lane's ring and its chunks' terminator masks in LDS.  (The masks in registers -- four per lane, read by
// bit-mask selects -- measured slower: the walker is bound by VALU issue, and a select costs more VALU than the
// LDS read it replaces; profiles/r05_walk/README.md.)
struct DWLds {
  // terminator mask of the chunk in each slot (bit i: byte i has its top bit clear), lane-major, slot 0 repeated as
  // slot DW_S: the masks of chunks k and k + 1 are adjacent, one ds_read2_b64
  uint64_t mask[WAVE][DW_S + 1];
  // YGM_DW_LM 1: lane l's ring is the 256 bytes at 256 l, its stream byte r at (r ^ 16 l) & 255 -- one v_bitop3 per
  // address (lanes reading the same stream offset land 16 bytes apart: spread over the banks);
  // 0: piece-major, piece p of lane l at (p * WAVE + l) * 16
  alignas(16) uint8_t ring[DW_P * WAVE * 16];
  uint32_t ordk[DW_BATCH];        // the current batch of documents, largest first: (min(bytes + 1, 2^24 - 1) << 8 | index in batch)
};                                // (one __shared__ object at LDS offset 0, masks first: their addresses need no
                                  // base add, the ring's base goes in the ds instructions' offset field)
// the masks of chunks k and k + 1
YDEV void dw_mask2(const DWLds& L, uint32_t l, uint32_t k, uint64_t& lo, uint64_t& hi) {
  const uint64_t* m = &L.mask[l][0] + (k & (DW_S - 1));
  lo = m[0]; hi = m[1];
}
// the same from a stream position r (chunk r >> 6): v_bfe + v_lshl_add for the address
YDEV void dw_mask2r(const DWLds& L, uint32_t l, uint32_t r, uint64_t& lo, uint64_t& hi) {
  const uint64_t* m = &L.mask[l][0] + __builtin_amdgcn_ubfe(r, 6, 2);
  lo = m[0]; hi = m[1];
}
static_assert(DW_S == 4, "dw_mask2r extracts a 2-bit slot");
static_assert(DW_S * 64 == 256 || !YGM_DW_LM, "the lane-major ring is 256 bytes per lane");
// LDS byte offset of stream byte r of lane l's ring
YDEV uint32_t dw_ra(uint32_t l, uint32_t r) {
#if YGM_DW_LM
  const uint32_t K = (l << 8) | ((l << 4) & 0xF0u);
  // (K & ~0xFF) | ((r ^ K) & 0xFF) as ONE v_bitop3 (M ? r ^ K : K, M = 0xFF; table index 4r + 2K + M: 0x6C) -- the
  // compiler splits the expression into a bitop3 and an add
  return __builtin_amdgcn_bitop3_b32(r, K, 0xFFu, 0x6C);
#else
  return (((r >> 4) & (DW_P - 1)) * WAVE + l) * 16u + (r & 15u);
#endif
}
YDEV u32x4& dw_piece(DWLds& L, uint32_t l, uint32_t r) { return *(u32x4*)(L.ring + dw_ra(l, r & ~15u)); }
YDEV const u32x4& dw_piece(const DWLds& L, uint32_t l, uint32_t r) { return *(const u32x4*)(L.ring + dw_ra(l, r & ~15u)); }

enum : uint32_t { WK_IDLE = 0, WK_SVN, WK_SVE, WK_UPD, WK_BLK, WK_ST, WK_STR, WK_DS, WK_DSC, WK_DSR, WK_FIN };

YDEV uint64_t dw_lowmask(uint32_t n) { return n >= 64u ? ~0ull : ((1ull << n) - 1ull); }
YDEV uint32_t dw_ctz(uint64_t x) { return x ? (uint32_t)__builtin_ctzll(x) : 64u; }
// bits >= p of x (p may be >= 64)
YDEV uint64_t dw_from(uint64_t x, uint32_t p) { return p >= 64u ? 0ull : (x >> p) << p; }
// (lo, hi) >> sh for sh in [0, 63]
YDEV uint64_t dw_fsh(uint64_t lo, uint64_t hi, uint32_t sh) { return (lo >> sh) | ((hi << (63u - sh)) << 1); }
// bytes of the varuint of v: 1 + floor(bits / 7) for bits = index of the top set bit ((x * 37) >> 8 == x / 7 for x < 64)
YDEV uint32_t dw_vulen(uint32_t v) { return 1u + (((31u - (uint32_t)__builtin_clz(v | 1u)) * 37u) >> 8); }

// the aligned 8 ring bytes at ring-relative x (x % 8 == 0)
YDEV uint64_t dw_word(const DWLds& L, uint32_t l, uint32_t x) { return *(const uint64_t*)(L.ring + dw_ra(l, x)); }
YDEV uint32_t dw_byte(const DWLds& L, uint32_t l, uint32_t r) { return L.ring[dw_ra(l, r)]; }
// 16 bytes at ring-relative r as (lo, hi)
YDEV void dw_rd16(const DWLds& L, uint32_t l, uint32_t r, uint64_t& lo, uint64_t& hi) {
  const uint32_t A = r & ~7u, sh = (r & 7u) * 8u;
  const uint64_t w0 = dw_word(L, l, A), w1 = dw_word(L, l, A + 8u), w2 = dw_word(L, l, A + 16u);
  lo = dw_fsh(w0, w1, sh);
  hi = dw_fsh(w1, w2, sh);
}
YDEV uint64_t dw_rd8(const DWLds& L, uint32_t l, uint32_t r) {
  const uint32_t A = r & ~7u;
  return dw_fsh(dw_word(L, l, A), dw_word(L, l, A + 8u), (r & 7u) * 8u);
}
// 8 bytes from byte p (p < 16) of the 16-byte view (lo, hi); bytes past the view read as 0
YDEV uint64_t dw_at(uint64_t lo, uint64_t hi, uint32_t p) { return p >= 8u ? (hi >> (8u * (p - 8u))) : dw_fsh(lo, hi, 8u * p); }
// 16 ring bytes at any alignment (for the output stream)
YDEV u32x4 dw_ring16(const DWLds& L, uint32_t l, uint32_t r) {
  const u32x4 a = dw_piece(L, l, r), b = dw_piece(L, l, r + 16u);
  const uint32_t s = (r >> 2) & 3u, sh = r & 3u;
  // dword s + j of (a, b) for j = 0..4 by bit-mask selects: a ?: over array elements is turned into a
  // scratch-indexed load by the compiler (one scratch round trip per copy-run head)
  const uint32_t m0 = 0u - (s & 1u), m1 = 0u - ((s >> 1) & 1u);
  auto sel4 = [&](uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) {   // d_s
    return bsel(m1, bsel(m0, d3, d2), bsel(m0, d1, d0));
  };
  const uint32_t E[5] = {sel4(a.x, a.y, a.z, a.w), sel4(a.y, a.z, a.w, b.x), sel4(a.z, a.w, b.x, b.y), sel4(a.w, b.x, b.y, b.z),
                         sel4(b.x, b.y, b.z, b.w)};
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(E[1], E[0], sh);
  o.y = __builtin_amdgcn_alignbyte(E[2], E[1], sh);
  o.z = __builtin_amdgcn_alignbyte(E[3], E[2], sh);
  o.w = __builtin_amdgcn_alignbyte(E[4], E[3], sh);
  return o;
}
// 64-bit terminator window at ring-relative r: bit i = byte r + i ends a varuint.  Chunks not yet
// landed read as "no terminator" (only used where the segment ends before them).
YDEV uint64_t dw_win(const DWLds& L, uint32_t l, uint32_t r, uint32_t landed) {
  const uint32_t k = r >> 6;
  uint64_t lo, hi;
  dw_mask2r(L, l, r, lo, hi);
  return dw_fsh(lo, k + 1u < landed ? hi : 0ull, r & 63u);
}
// value of the n-byte varuint (n = 1..5) in the low bytes of w; bad when n is outside 1..5 or >= 2^32
YDEV uint32_t dw_val(uint64_t w, uint32_t n, uint32_t& bad) {
  bad |= (n - 1u) > 4u ? 1u : 0u;
  const uint32_t nn = n > 5u ? 5u : (n ? n : 1u);
  bad |= (nn == 5u && ((w >> 32) & 0x70u)) ? 1u : 0u;
  return (uint32_t)pext7(w, nn);
}
// the bytes [p, p + 8) of the struct at q: from the 16-byte view when p <= 8, else from the ring
YDEV uint64_t dw_bytes_at(const DWLds& L, uint32_t l, uint32_t q, uint64_t lo, uint64_t hi, uint32_t p) {
  return p <= 8u ? dw_at(lo, hi, p) : dw_rd8(L, l, q + p);
}
// a varString at p of the unit at q (window win): returns the position after it; ASCII only, inside the window
YDEV uint32_t dw_str(const DWLds& L, uint32_t l, uint32_t q, uint64_t win, uint64_t lo, uint64_t hi, uint32_t p, uint32_t& bad) {
  const uint32_t e = dw_ctz(dw_from(win, p));
  const uint32_t n = dw_val(dw_bytes_at(L, l, q, lo, hi, p < 56u ? p : 56u), e - p + 1u, bad);
  const uint32_t s = e + 1u, f = s + n;
  bad |= f > 64u ? 1u : 0u;
  bad |= (s < 64u && ((~win >> s) & dw_lowmask(n))) ? 1u : 0u;
  return f;
}

// Writes a chunk to its ring slot and builds its terminator mask; checks the segment part
// [vlo, vhi) of it for varuints of >= 6 bytes (runs of >= 6 top-bit bytes: values past 2^35, which the
// walker never takes) and, with BP, for non-minimal varuints (a top-bit byte followed by a zero byte:
// yjs re-encodes them minimally, so a verbatim copy would differ -- diff only; the state vector is
// written from values), carrying the previous chunk's last 8 top bits in prev8.
template <bool BP>
YDEV void dw_commit(DWLds& L, uint32_t l, uint32_t k, const u32x4& p0, const u32x4& p1, const u32x4& p2, const u32x4& p3,
                    uint32_t vlo, uint32_t vhi, uint32_t& prev8, uint32_t& bad) {
  const uint32_t s = k & (DW_S - 1);
  dw_piece(L, l, 64u * k) = p0;
  dw_piece(L, l, 64u * k + 16u) = p1;
  dw_piece(L, l, 64u * k + 32u) = p2;
  dw_piece(L, l, 64u * k + 48u) = p3;
  const uint32_t D[16] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, p2.w, p3.x, p3.y, p3.z, p3.w};
  uint64_t H = 0, Z = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint32_t a = D[2 * j], b = D[2 * j + 1];
    H |= (uint64_t)hibits8(a, b) << (8 * j);
    if (BP) {
      const uint32_t za = ~(((a & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | a) & 0x80808080u;
      const uint32_t zb = ~(((b & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | b) & 0x80808080u;
      Z |= (uint64_t)hibits8(za, zb) << (8 * j);
    }
  }
  L.mask[l][s] = ~H;
  if (s == 0u) L.mask[l][DW_S] = ~H;
  const uint64_t vm = dw_lowmask(vhi) & ~dw_lowmask(vlo);
  const uint64_t Hm = H & vm;
  const uint64_t r2 = Hm & (Hm >> 1), r4 = r2 & (r2 >> 2), r6 = r4 & (r2 >> 4);
  const uint32_t c = ((uint32_t)(Hm & 0xFFu) << 8) | prev8;
  const uint32_t c2 = c & (c >> 1), c4 = c2 & (c2 >> 2), c6 = c4 & (c2 >> 4);
  uint64_t bp = 0;
  if (BP) bp = ((Hm << 1) | ((prev8 >> 7) & 1u)) & Z & vm;
  bad |= (bp | r6 | (uint64_t)c6) ? 1u : 0u;
  prev8 = (uint32_t)(Hm >> 56);
}

// the bytes of the varuint of v in the low bytes
YDEV uint64_t dw_vu_enc(uint32_t v) {
  const uint64_t x = (uint64_t)(v & 0x7Fu) | ((uint64_t)((v >> 7) & 0x7Fu) << 8) | ((uint64_t)((v >> 14) & 0x7Fu) << 16) |
                     ((uint64_t)((v >> 21) & 0x7Fu) << 24) | ((uint64_t)(v >> 28) << 32);
  return x | (0x8080808080ull & ((1ull << (8u * (dw_vulen(v) - 1u))) - 1ull));
}
// appends the varuint of v at byte `at` of the 16-byte value (lo, hi) (at + its length <= 16)
YDEV void dw_app(uint64_t& lo, uint64_t& hi, uint32_t& at, uint32_t v) {
  const uint64_t x = dw_vu_enc(v);
  if (at < 8u) { lo |= x << (8u * at); hi |= at ? x >> (64u - 8u * at) : 0ull; }
  else hi |= x << (8u * (at - 8u));
  at += dw_vulen(v);
}
// one 16-byte store at any alignment
YDEV void dw_st16(uint8_t* __restrict__ o, uint64_t lo, uint64_t hi) {
  u32x4 v;
  v.x = (uint32_t)lo; v.y = (uint32_t)(lo >> 32); v.z = (uint32_t)hi; v.w = (uint32_t)(hi >> 32);
  __builtin_memcpy(o, &v, 16);
}
// byte stores of a varuint at o[t..]; returns the new position
YDEV uint64_t dw_put_vu(uint8_t* __restrict__ o, uint64_t t, uint32_t v) {
  while (v > 127u) { o[t++] = (uint8_t)(0x80u | (v & 127u)); v >>= 7; }
  o[t++] = (uint8_t)v;
  return t;
}
}  // namespace ygm
