// ygm_merge_lean.hpp -- mergeUpdates fast path for Hocuspocus debounce logs: ONE WAVE PER
// DOCUMENT, no calls, no scratch, no per-struct LDS records.
//
// Shape it takes (the onChange stream of row a4/a5): k >= 2 updates of
// <= 32 bytes, each either ONE client block of Items (ContentString ASCII / ContentDeleted)
// or no structs at all (a deletion: delete set only), at most 4 distinct struct clients,
// every client's updates clock-contiguous in log order, and at most 64 delete-set ranges
// in the document.  For such a document rule R-M degenerates to:
// blocks by client descending, each block = the clients' structs in log order, copied
// byte for byte (Items never merge, Y@79424; no gaps, so no Skips; no GC, so no
// coalescing); the delete sets are unioned by rule R-DS (one range per lane: rank sort,
// segmented max scan, run encoding).  Anything else -- or anything
// this kernel cannot prove -- is deferred to the general kernels (k_merge_wave ->
// k_merge_fast -> k_merge_seq), which also produce every error status.
//
// Phases (all in registers except the two LDS byte buffers):
//   stage   every 16-byte chunk load of the document issued before the first wait
//   parse   lane per update (rows q = 0..3 hold updates l + 64q); the update's bytes are
//           read as three aligned ds_read_b128 and normalised to a 32-byte register
//           window; varuint ends come from a terminator bit mask (no byte loop)
//   clients distinct clients by wave vote, ranked descending (scalar)
//   scan    per-row DPP scans of packed 16-bit per-client byte counts; predecessor
//           clock checks by one bpermute per row
//   emit    ds_or_b32 of funnel-shifted source dwords into a zeroed LDS output buffer
//           (branch-free, order-free), then 16-byte coalesced stores
#pragma once
#include "ygm_common.hpp"
#include "ygm_merge_wave.hpp"

namespace ygm {

#ifndef YGM_LN_IN
#define YGM_LN_IN 5120
#endif
#ifndef YGM_LN_OUT
#define YGM_LN_OUT 4096
#endif
constexpr int LN_IN = YGM_LN_IN;     // staged input bytes (including the 0..15 byte alignment shift; a multiple of 16)
constexpr int LN_ROWS = 4;      // updates per lane: k <= 256
constexpr int LN_UMAX = 32;     // bytes per update
constexpr int LN_CMAX = 8;      // distinct struct clients per document

constexpr int LN_OUT = YGM_LN_OUT;    // staged output bytes

// The wide variant (k_merge_lean<1>, run over the documents the narrow one defers): updates of up to
// 64 bytes (multi-character inserts, SURVEY.md §8d's realistic debounce logs), documents of up to 7 KB
// staged, 6 KB of output (LDS 13.5 KB, <= 168 VGPRs: 3 waves per SIMD).
constexpr int LNW_IN = 7168;
constexpr int LNW_UMAX = 64;
constexpr int LNW_OUT = 6144;

template <int WIDE> struct LnCfg {
  static constexpr int IN = WIDE ? LNW_IN : LN_IN;
  static constexpr int OUT = WIDE ? LNW_OUT : LN_OUT;
  static constexpr int UMAX = WIDE ? LNW_UMAX : LN_UMAX;
};
#ifndef YGM_LN_INSLACK
#define YGM_LN_INSLACK 96
#endif
#ifndef YGM_LN_PAD
#define YGM_LN_PAD 0   // experiment only: LDS bytes added per wave (occupancy A/B, profiles/r06_lean)
#endif
template <int WIDE>
struct alignas(16) LeanLdsT {
  uint8_t in[LnCfg<WIDE>::IN + (WIDE ? 96 : YGM_LN_INSLACK)];   // + slack: window / copy reads reach up to 76 bytes past an update's start
  uint8_t out[LnCfg<WIDE>::OUT + 80 + (WIDE ? 0 : YGM_LN_PAD)];   // + slack: lds_or_copy ORs zero into up to 68 bytes past a range
};
static_assert(LN_IN % 16 == 0 && YGM_LN_INSLACK >= 80 && YGM_LN_INSLACK % 16 == 0, "staging granules and slack");
typedef LeanLdsT<0> LeanLds;

typedef __attribute__((address_space(3))) uint8_t LB8;
typedef __attribute__((address_space(3))) uint32_t LB32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 LB128;

// ---- DPP wave scans (row_shr within 16-lane rows, then row_bcast:15 / row_bcast:31)
YDEV uint32_t dpp_incl_add(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}
YDEV uint32_t dpp_incl_max(uint32_t x) {   // inclusive prefix max (unsigned); lane 63 holds the wave's max
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
  return x;
}
YDEV uint32_t lane63(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }
YDEV uint32_t rdlane(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); }
YDEV uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---- register window: bytes 0..39 of one update (U[0] = bytes 0..7)
// 8 bytes starting at byte p (p <= 31)
YDEV uint64_t win8(const uint64_t (&U)[5], uint32_t p) {
  const uint32_t q = p >> 3, sh = (p & 7u) * 8u;
  const uint64_t a01 = (q & 1) ? U[1] : U[0], a23 = (q & 1) ? U[3] : U[2];
  const uint64_t b12 = (q & 1) ? U[2] : U[1], b34 = (q & 1) ? U[4] : U[3];
  const uint64_t lo = (q & 2) ? a23 : a01, hi = (q & 2) ? b34 : b12;
  return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
}
YDEV uint32_t byte_at(const uint64_t (&U)[5], uint32_t p) { return (uint32_t)win8(U, p) & 0xFFu; }
// value of an n-byte varuint (1 <= n <= 8) whose bytes start the word w
YDEV uint64_t pext7(uint64_t w, uint32_t n) {
  uint64_t x = (n >= 8 ? w : (w & ((1ull << (8u * n)) - 1ull))) & 0x7f7f7f7f7f7f7f7full;
  x = ((x >> 1) & 0x3f803f803f803f80ull) | (x & 0x007f007f007f007full);
  x = ((x >> 2) & 0x0fffc0000fffc000ull) | (x & 0x00003fff00003fffull);
  x = ((x >> 4) & 0x00fffffff0000000ull) | (x & 0x000000000fffffffull);
  return x;
}
// 8 bits: bit i = top bit of byte i of the 8 bytes (lo, hi) -- two v_dot4_u32_u8, no multiplies
YDEV uint32_t hibits8(uint32_t lo, uint32_t hi) {
  const uint32_t a = __builtin_amdgcn_udot4((lo >> 7) & 0x01010101u, 0x08040201u, 0u, false);
  return __builtin_amdgcn_udot4((hi >> 7) & 0x01010101u, 0x80402010u, a, false);
}

// One parsed update (row record).
// staged position of an update's delete set: right after its structs (update at us, span of
// its parse), or after the 0 block count of an update without structs
YDEV uint32_t lean_ds_pos(uint32_t us, uint32_t span) { return span ? (span >> 16) + (span & 0xFFu) : us + 1u; }

struct LRec {
  uint32_t client, clock, clen;
  uint32_t span;   // sstart (doc-relative staged position of the first struct) << 16 | nst << 8 | sbytes
  bool ok;
};

// value of the <= 5-byte varuint whose first 4 bytes are x and 5th byte is y (n = length)
YDEV uint32_t pext32(uint32_t x, uint32_t y, uint32_t n) {
  x &= n >= 4u ? 0xFFFFFFFFu : ((1u << (8u * n)) - 1u);
  x &= 0x7f7f7f7fu;
  x = ((x >> 1) & 0x3f803f80u) | (x & 0x007f007fu);
  x = ((x >> 2) & 0x0fffc000u) | (x & 0x00003fffu);
  return x | (n >= 5u ? (y & 0x7Fu) << 28 : 0u);
}

// Parses the update at staged position s (n bytes).  ok == false: the document is deferred.
// Failure conditions are OR-ed into one integer (no per-condition lane masks); bytes the
// walk branches on (info, parentInfo, string lengths) are single ds_read_u8 of the staged
// copy; varuint ends come from the terminator mask T.
// bitwise select: x where m is set, y elsewhere (no ?: on array elements -- the compiler turns
// a ?: of array elements into a scratch-indexed load)
YDEV uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) { return (x & m) | (y & ~m); }

// W bytes (32 or 64) of staged input from position s as d[0..W/4): dword-aligned ds_read_b32
// funnelled by v_alignbyte (no selects; an unaligned b128 read replays)
template <int W>
YDEV void lean_windowW(LB8* in, uint32_t s, uint32_t (&d)[W / 4]) {
  const LB32* w = (const LB32*)(in + (s & ~3u));
  uint32_t L[W / 4 + 1];
#pragma unroll
  for (int j = 0; j <= W / 4; j++) L[j] = w[j];
#pragma unroll
  for (int j = 0; j < W / 4; j++) d[j] = __builtin_amdgcn_alignbyte(L[j + 1], L[j], s & 3u);
}
YDEV void lean_window(LB8* in, uint32_t s, uint32_t (&d)[8]) { lean_windowW<32>(in, s, d); }
// top bits of the 8 bytes (lo, hi) as bits 0..7: bytes masked to 0x00 / 0x80 times u8 weights
YDEV uint32_t top8(uint32_t lo, uint32_t hi) {
  const uint32_t a = __builtin_amdgcn_udot4(lo & 0x80808080u, 0x08040201u, 0u, false);
  return __builtin_amdgcn_udot4(hi & 0x80808080u, 0x80402010u, a, false) >> 7;
}
// the window's mask type: bit i <-> byte i
template <int W> struct LnMask;
template <> struct LnMask<32> { typedef uint32_t T; };
template <> struct LnMask<64> { typedef uint64_t T; };
// H = top-bit mask of the W window bytes
template <int W>
YDEV typename LnMask<W>::T lean_hmaskW(const uint32_t (&d)[W / 4]) {
  typename LnMask<W>::T H = 0;
#pragma unroll
  for (int j = 0; j < W / 8; j++) H |= (typename LnMask<W>::T)top8(d[2 * j], d[2 * j + 1]) << (8 * j);
  return H;
}
YDEV uint32_t lean_hmask(const uint32_t (&d)[8]) { return lean_hmaskW<32>(d); }
// index of the lowest set bit of x with the top bit forced (x == 0 -> W - 1)
YDEV uint32_t lnctz(uint32_t x) { return (uint32_t)__builtin_ctz(x | 0x80000000u); }
YDEV uint32_t lnctz(uint64_t x) { return (uint32_t)__builtin_ctzll(x | 0x8000000000000000ull); }

// Parses the update at staged position s (n bytes) from a W-byte register window (W = 32: the narrow
// kernel; 64: the wide one).  ok == false: the document is deferred.
template <int W>
YDEV LRec lean_parse(LB8* in, uint32_t s, uint32_t n) {
  typedef typename LnMask<W>::T M;
  constexpr uint32_t WB = (uint32_t)W, WL = WB - 1u;
  constexpr M ONE = 1, ALL = ~(M)0;
  LRec R; R.ok = false; R.client = 0; R.clock = 0; R.clen = 0; R.span = 0;
  if (n < 2 || n > WB) return R;
  uint32_t d[W / 4];
  lean_windowW<W>(in, s, d);
  if ((d[0] & 0xFFu) == 0u) { R.ok = true; return R; }   // no structs: a delete set only (at s + 1)
  // masks over the W window bytes: H = top bit set, Z = zero byte ("haszero": may also flag a
  // 0x01 right above a zero byte, which only defers)
  const M H = lean_hmaskW<W>(d);
  M Z = 0;
#pragma unroll
  for (int j = 0; j < W / 8; j++)
    Z |= (M)top8((d[2 * j] - 0x01010101u) & ~d[2 * j], (d[2 * j + 1] - 0x01010101u) & ~d[2 * j + 1]) << (8 * j);
  const M V = n >= WB ? ALL : ((ONE << n) - ONE);
  const M T = ~H & V;                 // varuint terminators among the valid bytes
  const M HV = H & V;
  LB8* u = in + s;
  // Whole-window checks instead of per-varuint ones:
  //  * a run of >= 7 bytes with the top bit set (a varuint of >= 8 bytes: possibly >= 2^53) defers;
  //  * a zero byte right after a top-bit byte is a non-minimal varuint terminator (or a client
  //    id 0 right after an info byte) -- yjs re-encodes those, so the document defers.
  const M h2 = HV & (HV >> 1), h4 = h2 & (h2 >> 2), h7 = h4 & (h4 >> 3);
  M bad = h7 | (Z & (HV << 1) & V);
  // position of the terminator of the varuint at p; past the window: >= WB-1 (then p >= n fails below)
#define LN_VEND(p, e) ((e) = ((p) < WL ? (p) : WL) + lnctz((M)(T >> ((p) < WL ? (p) : WL))))
  // ASCII run of L bytes at p inside the update (L < WB)
#define LN_ASCII(p, L) (bad |= (M)(((n - (p) - (L)) & 0x80000000u) | ((L) & ~WL)) | ((HV >> ((p) < WL ? (p) : WL)) & ((ONE << ((L) & WL)) - ONE)))
  const uint32_t b0 = d[0] & 0xFFu, b1 = (d[0] >> 8) & 0xFFu;
  bad |= (M)((b0 ^ 1u) | ((b1 - 1u) & ~127u) | (n < 4u ? 1u : 0u));    // one client block of 1..127 structs
  uint32_t e, p;
  LN_VEND(2u, e);
  const uint32_t cl_n = e - 1u;              // client bytes 2..e
  const uint32_t client = pext32(__builtin_amdgcn_alignbyte(d[1], d[0], 2u), (d[1] >> 16) & 0xFFu, cl_n);
  bad |= (M)((cl_n > 5u ? 1u : 0u) | (cl_n == 5u ? ((d[1] >> 16) & 0x70u) : 0u));   // clients are uint32
  p = e + 1u;                                 // 3..7
  LN_VEND(p, e);
  const uint32_t ck_n = e - p + 1u;
  const uint64_t U01 = ((uint64_t)d[1] << 32) | d[0], U23 = ((uint64_t)d[3] << 32) | d[2];
  const uint64_t cw = (U01 >> (8u * (p & 7u))) | (p & 7u ? (U23 << (64u - 8u * (p & 7u))) : 0ull);   // bytes p..p+7, 3 <= p <= 7
  const uint32_t clock = pext32((uint32_t)cw, (uint32_t)(cw >> 32) & 0xFFu, ck_n);
  bad |= (M)((ck_n > 5u ? 1u : 0u) | (ck_n == 5u ? ((uint32_t)(cw >> 32) & 0x70u) : 0u));
  p = e + 1u;
  const uint32_t sstart = p;
  uint32_t clen = 0;
  constexpr uint32_t PC = WB + 8u;            // byte reads clamp here (the staged buffer has slack)
  // structs: the first always, the rest (multi-struct transactions) by the back edge
  uint32_t st = 0;
  do {
    const uint32_t pc = p < PC ? p : PC;
    const uint32_t info = u[pc];
    p = pc + 1u;
    const uint32_t ref = info & 31u;
    // Skip/GC/other content go to the general path; bit 0x20 is dropped on re-encode when an origin is set
    bad |= (M)((info == 10u ? 1u : 0u) | ((ref != 1u && ref != 4u) ? 1u : 0u) | ((info & 0xC0u) && (info & 0x20u) ? 1u : 0u));
    // origin and/or right origin: 2 or 4 varuints -- the 2nd / 4th terminator from p
    {
      const uint32_t pp = p < WL ? p : WL;
      const M t0 = (T >> pp) | (ONE << WL), t1 = t0 & (t0 - ONE), t2 = t1 & (t1 - ONE), t3 = t2 & (t2 - ONE);
      const uint32_t nsk = ((info >> 6) & 1u) + ((info >> 7) & 1u);   // id pairs
      const uint32_t e2 = pp + lnctz(t1) + 1u;
      const uint32_t e4 = pp + lnctz(t3) + 1u;
      p = nsk == 2u ? e4 : nsk == 1u ? e2 : p;
    }
    if ((info & 0xC0u) == 0u) {   // parent (rare: inserts at the start of a type, map keys)
      const uint32_t pi = u[p < PC ? p : PC]; p++;
      if (pi == 1u) {
        const uint32_t Lk = u[p < PC ? p : PC]; p++;
        LN_ASCII(p, Lk); p += Lk & WL;
      } else {
        bad |= (M)pi;                  // parentInfo is re-encoded as 0/1
        LN_VEND(p, e); p = e + 1u; LN_VEND(p, e); p = e + 1u;
      }
      if (info & 0x20u) {
        const uint32_t Ls = u[p < PC ? p : PC]; p++;
        LN_ASCII(p, Ls); p += Ls & WL;
      }
    }
    if (ref == 1u) {   // ContentDeleted: varuint length
      LN_VEND(p, e);
      const uint32_t pp = p < WL ? p : WL;
      const uint32_t x = u[pp] | ((uint32_t)u[pp + 1] << 8) | ((uint32_t)u[pp + 2] << 16) | ((uint32_t)u[pp + 3] << 24);
      const uint32_t v = pext32(x, 0u, e - p + 1u);
      bad |= (M)((v == 0u ? 1u : 0u) | ((e - p) > 2u ? 1u : 0u));   // 1..3 bytes: < 2^21
      clen += v;
      p = e + 1u;
    } else {           // ContentString: single-byte length, ASCII bytes (UTF-16 length == byte length)
      const uint32_t Lc = u[p < PC ? p : PC]; p++;
      bad |= (M)(Lc == 0u ? 1u : 0u);
      LN_ASCII(p, Lc);
      p += Lc & WL;
      clen += Lc;
    }
  } while (++st < b1 && (bad | (M)(p >= n ? 1u : 0u)) == 0);
#undef LN_VEND
#undef LN_ASCII
  bad |= (M)((n - 1u - p) & 0x80000000u);          // then the delete set (at least its count byte)
  bad |= (M)(uint32_t)(((uint64_t)clock + clen) >> 32);
  R.ok = bad == 0;
  R.client = client; R.clock = clock; R.clen = clen;
  R.span = ((s + sstart) << 16) | (b1 << 8) | ((p - sstart) & 0xFFu);   // the delete set follows the structs
  return R;
}

// byte p (0..31) of a 32-byte register window.  Selects by bit masks (v_bfi): a ?: over array elements is
// turned into a scratch-indexed load by the compiler
YDEV uint32_t w2_byte(const uint32_t (&d)[8], uint32_t p) {
  const uint32_t i = p >> 2;
  const uint32_t m0 = 0u - (i & 1u), m1 = 0u - ((i >> 1) & 1u), m2 = 0u - ((i >> 2) & 1u);
  const uint32_t a0 = bsel(m0, d[1], d[0]), a1 = bsel(m0, d[3], d[2]), a2 = bsel(m0, d[5], d[4]), a3 = bsel(m0, d[7], d[6]);
  const uint32_t b0 = bsel(m1, a1, a0), b1 = bsel(m1, a3, a2);
  return (bsel(m2, b1, b0) >> (8u * (p & 3u))) & 0xFFu;
}
// bytes [p, p + 5) of a register window, p <= 15, as (the first 4 bytes, the 5th byte)
YDEV void w2_vu5(const uint32_t (&d)[8], uint32_t p, uint32_t& x, uint32_t& y) {
  const uint32_t i = p >> 2, s = p & 3u;
  const uint32_t m0 = 0u - (i & 1u), m1 = 0u - ((i >> 1) & 1u);
  const uint32_t lo = bsel(m1, bsel(m0, d[3], d[2]), bsel(m0, d[1], d[0]));
  const uint32_t hi = bsel(m1, bsel(m0, d[4], d[3]), bsel(m0, d[2], d[1]));
  const uint32_t hh = bsel(m1, bsel(m0, d[5], d[4]), bsel(m0, d[3], d[2]));
  x = __builtin_amdgcn_alignbyte(hi, lo, s);
  y = __builtin_amdgcn_alignbyte(hh, hi, s) & 0xFFu;
}

// ---- delete sets (rule R-DS): a DS is varuints only, so one update's DS is
// walked in a 32-byte register window by its terminator mask, one range per call.
constexpr int LN_DSMAX = 64;    // delete-set ranges per document (one per lane in the union)
struct LDsCur {
  LB8* u;                       // the DS bytes (staged)
  uint32_t T, lim;              // terminator mask over the valid window bytes; window bytes of the update
  uint32_t p, cl_left, r_left, client, bad;
};
// next varuint of the DS (at most maxb bytes; 5 = any uint32): its end from the terminator
// mask, its bytes by independent ds_read_u8
YDEV uint32_t lean_ds_vu(LDsCur& c, uint32_t maxb) {
  const uint32_t pp = c.p < 31u ? c.p : 31u;
  const uint32_t e = pp + (uint32_t)__builtin_ctz((c.T >> pp) | 0x80000000u);
  const uint32_t nb = e - c.p + 1u;
  LB8* b = c.u + pp;
  const uint32_t x = b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24), y = b[4];
  c.bad |= (c.p >= c.lim ? 1u : 0u) | (e >= c.lim ? 1u : 0u) | (nb > maxb ? 1u : 0u) | (nb == 5u ? (y & 0x70u) : 0u);
  c.p = e + 1u;
  return pext32(x, y, nb);
}
// opens the DS at staged position a, n bytes to the end of its update
YDEV void lean_ds_open(LB8* in, uint32_t a, uint32_t n, LDsCur& c) {
  uint32_t d[8];
  lean_window(in, a, d);
  c.u = in + a;
  c.lim = n < 32u ? n : 32u;
  c.T = ~lean_hmask(d) & (c.lim >= 32u ? 0xFFFFFFFFu : ((1u << c.lim) - 1u));
  c.p = 0; c.bad = 0; c.r_left = 0; c.client = 0;
  c.cl_left = lean_ds_vu(c, 4u);
}
YDEV bool lean_ds_more(const LDsCur& c) { return c.bad == 0u && (c.r_left | c.cl_left) != 0u; }
// next range (client, clock, len); clients with no ranges defer (they add no records, but
// need a loop here); clocks and lengths below 2^28
YDEV void lean_ds_next(LDsCur& c, uint32_t& client, uint32_t& clock, uint32_t& len) {
  if (c.r_left == 0u) {
    c.client = lean_ds_vu(c, 5u);
    c.r_left = lean_ds_vu(c, 4u);
    c.bad |= c.r_left == 0u ? 1u : 0u;
    c.cl_left--;
  }
  client = c.client;
  clock = lean_ds_vu(c, 4u);
  len = lean_ds_vu(c, 4u);
  c.r_left -= c.r_left ? 1u : 0u;
}

// Copies n (4..31) bytes from staged input position s to output position t (both LDS) into a
// ZEROED output buffer: every destination dword the range touches gets ds_or_b32 of the
// funnel-shifted source bytes masked to the range.  Byte ranges of different lanes are
// disjoint, so the ORs commute: no edge cases, no ordering between lanes.  ND (wave-uniform)
// bounds the destination dwords: head + n <= 4 ND (lean_copy picks 6 or 9).
template <int ND>
YDEV void lds_or_copy(LB8* out, LB8* in, uint32_t t, uint32_t s, uint32_t n) {
  const uint32_t head = t & 3u;
  const uint32_t src0 = s - head;                 // source byte that maps to destination byte t & ~3
  const uint32_t sb = src0 & 3u;
  LB32* sw = (LB32*)(in + (src0 & ~3u));
  uint32_t w[ND + 1];
#pragma unroll
  for (int j = 0; j <= ND; j++) w[j] = sw[j];     // may read past the update: the staged buffer has slack
  LB32* od = (LB32*)(out + (t & ~3u));
  const uint32_t last = head + n;                 // destination bytes [head, last) of the dword run are ours
  const uint32_t jl = (last - 1u) >> 2;           // last dword touched
  const uint32_t mtail = 0xFFFFFFFFu >> (8u * (4u * jl + 4u - last));
#pragma unroll
  for (int j = 0; j < ND; j++) {
    const uint32_t v = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sb);
    uint32_t m = (uint32_t)j < jl ? 0xFFFFFFFFu : (uint32_t)j == jl ? mtail : 0u;
    if (j == 0) m &= 0xFFFFFFFFu << (8u * head);
    __hip_atomic_fetch_or(od + j, v & m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
// one row of struct copies: 6 destination dwords when every lane's run fits (C2 structs are
// <= 19 bytes), else 9, else (the wide kernel's runs of up to 63 bytes) 17
template <int WIDE>
YDEV void lean_copy(LB8* out, LB8* in, bool go, uint32_t t, uint32_t s, uint32_t n) {
  if (__ballot(go && (t & 3u) + n > 24u) == 0) { if (go) lds_or_copy<6>(out, in, t, s, n); }
  else if (!WIDE || __ballot(go && (t & 3u) + n > 36u) == 0) { if (go) lds_or_copy<9>(out, in, t, s, n); }
  else if (go) lds_or_copy<17>(out, in, t, s, n);
}
YDEV uint32_t lds_vu(LB8* out, uint32_t t, uint32_t v) {
  while (v > 127u) { out[t++] = (uint8_t)(0x80u | (v & 127u)); v >>= 7; }
  out[t++] = (uint8_t)v;
  return t;
}

YDEV uint32_t vlen32(uint32_t v) {   // bytes of the varuint encoding of v
  return 1u + (v > 0x7Fu ? 1u : 0u) + (v > 0x3FFFu ? 1u : 0u) + (v > 0x1FFFFFu ? 1u : 0u) + (v > 0xFFFFFFFu ? 1u : 0u);
}
// one DPP step of a 64-bit inclusive max scan: (hi, lo) pairs move together (lanes the pattern does not
// reach read (0, 0), which never wins)
template <int CTRL, int RM, bool BC>
YDEV void dpp_max64_step(uint32_t& hi, uint32_t& lo) {
  const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, RM, 0xF, BC);
  const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, RM, 0xF, BC);
  const bool gt = h2 > hi || (h2 == hi && l2 > lo);
  hi = gt ? h2 : hi; lo = gt ? l2 : lo;
}
// lane l's value of x at lane l ^ J (J = 1, 2: quad permutes; 4, 8: row shifts by lane bit; 16, 32: bpermute)
template <int J>
YDEV uint32_t lane_xor(uint32_t x) {
  if (J == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  if (J == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  if (J == 4 || J == 8) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 | J, 0xF, 0xF, false);   // row_shl:J (lane + J)
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 | J, 0xF, 0xF, false);   // row_shr:J (lane - J)
    return (threadIdx.x & J) ? dn : up;
  }
  return (uint32_t)__shfl_xor((int)x, J, 64);
}
// one compare-exchange stage of a 64-lane bitonic sort (ascending) on the key (a, b, c)
template <int K, int J>
YDEV void bitonic_step(uint32_t& a, uint32_t& b, uint32_t& c) {
  const uint32_t oa = lane_xor<J>(a), ob = lane_xor<J>(b), oc = lane_xor<J>(c);
  const bool lt = oa < a || (oa == a && (ob < b || (ob == b && oc < c)));   // other < mine
  const uint32_t l = threadIdx.x;
  const bool lower = (l & J) == 0, asc = (l & K) == 0;
  const bool take = lower == asc ? lt : !lt;   // the lower lane of an ascending pair keeps the minimum
  a = take ? oa : a; b = take ? ob : b; c = take ? oc : c;
}
template <int K, int J>
YDEV void bitonic_merge(uint32_t& a, uint32_t& b, uint32_t& c) {
  bitonic_step<K, J>(a, b, c);
  if constexpr (J > 1) bitonic_merge<K, J / 2>(a, b, c);
}
// sorts the 64 lanes' distinct keys (a, b, c) ascending: lane l gets the l-th smallest
YDEV void lane_bitonic3(uint32_t& a, uint32_t& b, uint32_t& c) {
  bitonic_merge<2, 1>(a, b, c);
  bitonic_merge<4, 2>(a, b, c);
  bitonic_merge<8, 4>(a, b, c);
  bitonic_merge<16, 8>(a, b, c);
  bitonic_merge<32, 16>(a, b, c);
  bitonic_merge<64, 32>(a, b, c);
}
YDEV uint64_t lean_max_scan64(uint64_t v) {   // inclusive prefix max over the wave (DPP, as dpp_incl_max)
  uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  dpp_max64_step<0x111, 0xF, true>(hi, lo);   // row_shr:1
  dpp_max64_step<0x112, 0xF, true>(hi, lo);   // row_shr:2
  dpp_max64_step<0x114, 0xF, true>(hi, lo);   // row_shr:4
  dpp_max64_step<0x118, 0xF, true>(hi, lo);   // row_shr:8
  dpp_max64_step<0x142, 0xA, false>(hi, lo);  // row_bcast:15 -> rows 1, 3
  dpp_max64_step<0x143, 0xC, false>(hi, lo);  // row_bcast:31 -> rows 2, 3
  return ((uint64_t)hi << 32) | lo;
}

// The merged delete set of one document (mergeDeleteSets Y@10486 + sortAndMergeDeleteSet
// Y@10246 + writeDeleteSet): lane i holds the i-th range of the union, sorted by (client
// descending, clock); the caller emits it with lean_ds_emit after zeroing the output buffer.
struct LDsUnion {
  uint32_t client, nruns, sclock, rend;   // per lane: its client / runs of its client / its run
  bool segstart, runend;
  uint32_t pos;                           // lane's first byte, relative to the DS start
  uint32_t nsegs, bytes;                  // uniform: clients, encoded DS bytes
  bool bad;
};
#ifdef YGM_DIAG
// diagnostic build: shader cycles of the union's parts (records, rank sort, runs / scans), summed over waves
static __device__ unsigned long long ygm_diag_ds[4];
#define LDS_T0 unsigned long long _dst = __builtin_amdgcn_s_memtime();
#define LDS_STAMP(i) do { const unsigned long long _n = __builtin_amdgcn_s_memtime(); if (threadIdx.x == 0) atomicAdd(&ygm_diag_ds[i], _n - _dst); _dst = _n; } while (0)
#else
#define LDS_T0
#define LDS_STAMP(i)
#endif
// scratch: 16 * LN_DSMAX bytes of LDS (records, then the sorted records)
YDEV LDsUnion lean_ds_union(LB8* lin, LB32* scr, const uint32_t (&dpos)[LN_ROWS], const uint32_t (&uend)[LN_ROWS],
                            const bool (&hasd)[LN_ROWS], uint32_t flags) {
  const uint32_t l = threadIdx.x;
  LDsUnion U; U.bad = false; U.nsegs = 0; U.bytes = 1; U.segstart = false; U.runend = false; U.pos = 0;
  U.client = 0; U.nruns = 0; U.sclock = 0; U.rend = 0;
  LB32* rc = scr; LB32* rk = scr + LN_DSMAX; LB32* re = scr + 2 * LN_DSMAX;
  LB32* rn = scr + 3 * LN_DSMAX;   // yjs 13.5 only: the record's first-seen rank (update << 8 | range index in it)
  uint32_t nrec = 0, bad = 0;
  LDS_T0
  // ---- records of every update's DS, in update order (the order only matters for ties, which
  //      the union does not see)
#pragma unroll
  for (int q = 0; q < LN_ROWS; q++) {
    if (__ballot(hasd[q]) == 0) continue;
    // fast path: a delete set of one client with one range (a deletion's update) -- its five varuint ends
    // from the terminator mask, the values from the register window, no dependent cursor walk
    bool fq = false;
    uint32_t fcl = 0, fck = 0, fln = 0;
    if (hasd[q]) {
      uint32_t w[8];
      lean_window(lin, dpos[q], w);
      const uint32_t n = uend[q] - dpos[q], lim = n < 32u ? n : 32u;
      const uint32_t T = ~lean_hmask(w) & (lim >= 32u ? 0xFFFFFFFFu : ((1u << lim) - 1u));
      const uint32_t t1 = T & (T - 1u), t2 = t1 & (t1 - 1u), t3 = t2 & (t2 - 1u), t4 = t3 & (t3 - 1u);
      const uint32_t e1 = lnctz(T), e2 = lnctz(t1), e3 = lnctz(t2), e4 = lnctz(t3), e5 = lnctz(t4);
      uint32_t cx, cy, kx, ky, lx, ly;
      w2_vu5(w, 1u, cx, cy);
      w2_vu5(w, (e3 + 1u) & 15u, kx, ky);
      w2_vu5(w, (e4 + 1u) & 15u, lx, ly);
      const uint32_t ncb = e2 - e1, nkb = e4 - e3, nlb = e5 - e4;   // bytes of client, clock, length
      fq = e1 == 0u && (w[0] & 0xFFu) == 1u && e3 == e2 + 1u && w2_byte(w, e3 & 31u) == 1u && e5 < lim &&
           ncb - 1u <= 4u && !(ncb == 5u && (cy & 0x70u)) && nkb - 1u <= 3u && nlb - 1u <= 3u;
      fcl = pext32(cx, cy, ncb); fck = pext32(kx, ky, nkb); fln = pext32(lx, ly, nlb);
    }
    {
      const uint64_t m = __ballot(fq);
      const uint32_t slot = nrec + lanes_below(m);
      if (fq && slot < (uint32_t)LN_DSMAX) { rc[slot] = fcl; rk[slot] = fck; re[slot] = fck + fln; rn[slot] = (l + 64u * q) << 8; }
      nrec += (uint32_t)__builtin_popcountll(m);
    }
    const bool slow = hasd[q] && !fq;
    if (__ballot(slow) == 0) continue;
    LDsCur c;
    if (slow) lean_ds_open(lin, dpos[q], uend[q] - dpos[q], c);
    else { c.bad = 0; c.cl_left = 0; c.r_left = 0; }
    for (int it = 0; it < LN_DSMAX; it++) {
      bool has = lean_ds_more(c);
      if (__ballot(has) == 0) break;
      uint32_t cl = 0, ck = 0, ln = 0;
      if (has) lean_ds_next(c, cl, ck, ln);
      has = has && c.bad == 0u;
      const uint64_t m = __ballot(has);
      const uint32_t slot = nrec + lanes_below(m);
      if (has && slot < (uint32_t)LN_DSMAX) { rc[slot] = cl; rk[slot] = ck; re[slot] = ck + ln; rn[slot] = ((l + 64u * q) << 8) | (uint32_t)it; }
      nrec += (uint32_t)__builtin_popcountll(m);
    }
    bad |= c.bad | (lean_ds_more(c) ? 1u : 0u);   // malformed, or more ranges than the loop takes
  }
  U.bad = __ballot(bad != 0u) != 0 || nrec > (uint32_t)LN_DSMAX || nrec == 0u;
  LDS_STAMP(0);
  if (U.bad) return U;
  wave_sync();
  // ---- sort by (client descending, clock ascending, record order): a register bitonic network over the
  //      64 lanes on the key (~client, clock, record index); empty lanes carry the largest key
  const bool v = l < nrec;
  uint32_t k0 = v ? ~rc[l] : 0xFFFFFFFFu, k1 = v ? rk[l] : 0xFFFFFFFFu, k2 = v ? l : 0xFFu;
  lane_bitonic3(k0, k1, k2);
  LDS_STAMP(1);
  // lane l holds the l-th record of the union order; its end from the record table (re is not rewritten)
  uint32_t c = v ? ~k0 : 0u, k = v ? k1 : 0u, e = v ? re[k2 & (LN_DSMAX - 1)] : 0u;
  if (flags & 1u) {
    // yjs 13.5.16 writes the merged delete set's clients in first-seen order (mergeDeleteSets' Map insertion order:
    // the first update holding the client, its position in that update's delete set; Y@10486, Y@11105).  Each
    // client's rank is the least rank of its records; the records are sorted again by (rank, clock, record) --
    // clients stay contiguous, so the runs below are the same, in that order.
    const uint32_t cp0 = (uint32_t)__shfl_up((int)c, 1u, 64);
    const bool ss0 = v && (l == 0u || cp0 != c);
    const uint32_t si0 = dpp_incl_add(ss0 ? 1u : 0u);   // (1-based) client segment of the lane
    const uint64_t mx = lean_max_scan64(v ? (((uint64_t)si0 << 32) | (uint32_t)~rn[k2 & (LN_DSMAX - 1)]) : 0ull);
    const bool nss0 = __shfl_down(ss0 ? 1 : 0, 1u, 64) != 0;
    const bool se0 = v && (l + 1u == nrec || nss0);   // the segment's last lane holds its least rank
    LB32* T = rk;                                      // (rk is not read after the sort: the clock is in the key)
    wave_sync();
    if (se0) T[si0 - 1u] = ~(uint32_t)mx;
    wave_sync();
    uint32_t s0 = v ? T[si0 - 1u] : 0xFFFFFFFFu, s1 = v ? k : 0xFFFFFFFFu, s2 = v ? k2 : 0xFFu;
    lane_bitonic3(s0, s1, s2);
    c = v ? rc[s2 & (LN_DSMAX - 1)] : 0u; k = v ? s1 : 0u; e = v ? re[s2 & (LN_DSMAX - 1)] : 0u;
    wave_sync();   // (rc is rewritten below)
  }
  const uint32_t cprev = (uint32_t)__shfl_up((int)c, 1u, 64);
  // ---- runs: a range starts a run when it is its client's first or starts past every end so far
  const bool segstart = v && (l == 0u || cprev != c);
  const uint32_t segidx = dpp_incl_add(segstart ? 1u : 0u);
  const uint32_t nsegs = lane63(segidx);
  const uint64_t incl = lean_max_scan64(v ? (((uint64_t)segidx << 32) | e) : 0ull);
  const uint32_t prevmax = (uint32_t)__shfl_up(incl, 1u, 64);
  const bool runstart = v && (segstart || k > prevmax);
  const bool nxt_rs = __shfl_down(runstart ? 1 : 0, 1u, 64) != 0;
  const bool runend = v && (l + 1u == nrec || nxt_rs);
  const uint32_t sidx = (uint32_t)lean_max_scan64(runstart ? l : 0u);
  const uint32_t sclock = (uint32_t)__shfl(k, (int)sidx, 64);
  // runs per client: the inclusive run count at the client's last range, minus the count before its first
  const uint32_t rsc = dpp_incl_add(runstart ? 1u : 0u);
  // (shuffles run with every lane active: a bpermute from an inactive lane reads 0)
  const bool nxt_ss = __shfl_down(segstart ? 1 : 0, 1u, 64) != 0;
  const bool segend = v && (l + 1u == nrec || nxt_ss);
  LB32* cnt = scr;                 // rc is free again
  wave_sync();
  if (segend) cnt[segidx - 1u] = rsc;
  wave_sync();
  const uint32_t nruns = segstart ? cnt[segidx - 1u] - rsc + 1u : 0u;
  const uint32_t tb = (segstart ? vlen32(c) + vlen32(nruns) : 0u) + (runend ? vlen32(sclock) + vlen32((uint32_t)incl - sclock) : 0u);
  const uint32_t ib = dpp_incl_add(tb);
  U.client = c; U.nruns = nruns; U.sclock = sclock; U.rend = (uint32_t)incl;
  U.segstart = segstart; U.runend = runend; U.pos = ib - tb;
  U.nsegs = nsegs; U.bytes = vlen32(nsegs) + lane63(ib);
  LDS_STAMP(2);
  return U;
}
// writes the delete set at t (the output buffer is zeroed)
YDEV void lean_ds_emit(LB8* out, uint32_t t, const LDsUnion& U) {
  if (threadIdx.x == 0) lds_vu(out, t, U.nsegs);
  uint32_t o = t + vlen32(U.nsegs) + U.pos;
  if (U.segstart) { o = lds_vu(out, o, U.client); o = lds_vu(out, o, U.nruns); }
  if (U.runend) { o = lds_vu(out, o, U.sclock); lds_vu(out, o, U.rend - U.sclock); }
}

}  // namespace ygm
