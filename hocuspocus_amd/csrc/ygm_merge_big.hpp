// ygm_merge_big.hpp -- mergeUpdates for LARGE [snapshot, ...log] documents:
// ONE WAVE PER DOCUMENT, global memory, no per-struct records for the snapshot.
//
// Shape it takes (what Hocuspocus stores: the engine's previous output plus the onChange updates
// since, row a4): the largest update U0 (the snapshot) has its client blocks in strictly
// descending client order and a delete set sorted by (client descending, clock); every other
// update (the log) is small -- at most LB_MAXS structs and LB_MAXD delete ranges in all -- has its
// blocks in descending client order too (else yjs's writer can revisit a client: golden vector
// 7955), and its structs do not overlap U0's or each other's clock ranges.  For that class rule R-M (SURVEY.md
// App. B.5) is: per client (descending), the pieces -- U0's block as one piece, every log struct
// as one piece -- in clock order, a Skip over every gap, U0's block bytes verbatim; and the delete
// sets are unioned by R-DS with U0's sorted list streamed.  Anything else (overlaps, input Skips,
// GC-GC junctions between sources, re-encoded structs, ContentDoc in U0, 13.5
// multi-client delete sets, malformed input) is deferred to the exact sequential kernel.
//
//   walk   lane 0 walks U0 with a 16-byte register-window cursor (GCur): every struct is validated
//          as read_struct does (UTF-8 by 16-byte chunks with an ASCII fast path) and must be
//          byte-for-byte what write_struct would emit; one table entry per block in global scratch
//   log    lanes walk the log updates in parallel (Cur over global memory; they are small) into
//          LDS records; bitonic sorts by (client descending, clock)
//   emit   lane 0 merges the block table with the sorted log pieces twice (sizes, then bytes);
//          the wave copies each U0 block range with 16-byte loads / stores
#pragma once
#include <type_traits>
#include "ygm_seqdoc.hpp"
#include "ygm_merge_lean.hpp"

namespace ygm {

constexpr int LB_MAXS = 1024;   // log structs per document
constexpr int LB_MAXD = 1024;   // log delete-set ranges per document

// ---- global-memory cursor with a 16-byte register window
struct GCur {
  const uint8_t* p;
  uint32_t pos, end;
  int err, nm;
  uintptr_t wa;                  // absolute address of the window (16-byte aligned); 1 = none
  uint32_t w0, w1, w2, w3;
  YDEV void init(const uint8_t* base, uint32_t n) { p = base; pos = 0; end = n; err = 0; nm = 0; wa = 1; }
  YDEV const uint8_t* gp() const { return p; }   // the bytes through a generic pointer (content checks)
  YDEV void fail(int e) { if (!err) err = e; pos = end; }
  YDEV uint32_t raw(uint32_t q) {        // byte at p + q (q < end: the aligned chunk is inside the arena)
    const uint8_t* ap = p + q;
    const uintptr_t a = (uintptr_t)ap, b = a & ~(uintptr_t)15;
    if (b != wa) {   // pointer arithmetic keeps the global address space (an integer round trip would make it flat)
      const uint4 v = *(const uint4*)(ap - (a & 15u));
      w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w; wa = b;
    }
    // selects between computed halves, not between the members: a select of two member loads becomes a
    // load through a selected pointer, and the cursor then cannot live in registers (scratch round trips)
    const uint32_t o = (uint32_t)(a & 15u);
    const uint64_t X = ((uint64_t)w1 << 32) | w0, Y = ((uint64_t)w3 << 32) | w2;
    const uint64_t h = (o & 8u) ? Y : X;
    return (uint32_t)(h >> (8u * (o & 7u))) & 0xFFu;
  }
  YDEV uint32_t u8() { if (pos >= end) { fail(ST_MALFORMED); return 0; } return raw(pos++); }
  YDEV uint64_t vu() {   // lib0 readVarUint (Cur::vu semantics)
    // fast path: the whole varuint (<= 8 bytes) inside the current 16-byte window and the update
    if (pos < end) {
      raw(pos);
      const uint32_t o = (uint32_t)(((uintptr_t)(p + pos)) & 15u);
      const uint64_t X = ((uint64_t)w1 << 32) | w0, Y = ((uint64_t)w3 << 32) | w2;
      const uint64_t v8 = o == 0 ? X : o < 8 ? (X >> (8 * o)) | (Y << (64 - 8 * o)) : (Y >> (8 * (o - 8)));
      const uint64_t t = ~v8 & 0x8080808080808080ull;
      const uint32_t k = t ? (uint32_t)__builtin_ctzll(t) >> 3 : 8u;          // terminator byte index
      if (k < 8u && k < 16u - o && pos + k < end) {
        const uint64_t num = pext7(v8, k + 1);
        if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
        if (k > 0 && ((v8 >> (8 * k)) & 0xFFu) == 0) nm = 1;
        pos += k + 1;
        return num;
      }
    }
    uint64_t num = 0; uint32_t shift = 0;
    for (;;) {
      if (pos >= end) { fail(ST_MALFORMED); return 0; }
      const uint32_t r = raw(pos++);
      if (shift < 63) num |= (uint64_t)(r & 127u) << shift;
      else if (r & 127u) { fail(ST_RANGE); return 0; }
      shift += 7;
      if (r < 128u) {
        if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
        if (r == 0 && shift > 7) nm = 1;
        return num;
      }
      if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
    }
  }
  YDEV uint32_t buf(uint32_t& len) {
    const uint64_t n = vu();
    if (err) { len = 0; return pos; }
    if (n > (uint64_t)(end - pos)) { fail(ST_MALFORMED); len = 0; return pos; }
    const uint32_t s = pos; pos += (uint32_t)n; len = (uint32_t)n; return s;
  }
};

// ---- the same cursor over bytes staged in LDS (the snapshot scan's stage): LDS-typed reads (ds_read, not flat loads
// through a generic pointer), a varuint from one 8-byte view built of three aligned dwords.  Reads reach 11 bytes
// past `end` (the stage's slack).
struct LCur {
  LU8* p;
  uint32_t pos, end;
  int err, nm;
  YDEV void init(LU8* base, uint32_t n) { p = base; pos = 0; end = n; err = 0; nm = 0; }
  YDEV const uint8_t* gp() const { return (const uint8_t*)p; }
  YDEV void fail(int e) { if (!err) err = e; pos = end; }
  YDEV uint32_t raw(uint32_t q) const { return p[q]; }
  YDEV uint64_t w8(uint32_t q) const {   // the 8 bytes at p + q
    const uint32_t a = (uint32_t)(uintptr_t)(p + q), sh = a & 3u;
    const __attribute__((address_space(3))) uint32_t* d = (const __attribute__((address_space(3))) uint32_t*)(p + q - sh);
    const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
    return ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32) | __builtin_amdgcn_alignbyte(d1, d0, sh);
  }
  YDEV void w16(uint32_t q, uint64_t& lo, uint64_t& hi) const {   // the 16 bytes at p + q
    const uint32_t a = (uint32_t)(uintptr_t)(p + q), sh = a & 3u;
    const __attribute__((address_space(3))) uint32_t* d = (const __attribute__((address_space(3))) uint32_t*)(p + q - sh);
    const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
    lo = ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32) | __builtin_amdgcn_alignbyte(d1, d0, sh);
    hi = ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, sh) << 32) | __builtin_amdgcn_alignbyte(d3, d2, sh);
  }
  YDEV uint32_t u8() { if (pos >= end) { fail(ST_MALFORMED); return 0; } return raw(pos++); }
  YDEV uint64_t vu() {   // lib0 readVarUint (Cur::vu semantics)
    if (pos < end) {
      const uint64_t v8 = w8(pos);
      const uint64_t t = ~v8 & 0x8080808080808080ull;
      const uint32_t k = t ? (uint32_t)__builtin_ctzll(t) >> 3 : 8u;   // terminator byte index
      if (k < 8u && pos + k < end) {
        const uint64_t num = pext7(v8, k + 1);
        if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
        if (k > 0 && ((v8 >> (8 * k)) & 0xFFu) == 0) nm = 1;
        pos += k + 1;
        return num;
      }
    }
    uint64_t num = 0; uint32_t shift = 0;
    for (;;) {
      if (pos >= end) { fail(ST_MALFORMED); return 0; }
      const uint32_t r = raw(pos++);
      if (shift < 63) num |= (uint64_t)(r & 127u) << shift;
      else if (r & 127u) { fail(ST_RANGE); return 0; }
      shift += 7;
      if (r < 128u) {
        if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
        if (r == 0 && shift > 7) nm = 1;
        return num;
      }
      if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
    }
  }
  YDEV uint32_t buf(uint32_t& len) {
    const uint64_t n = vu();
    if (err) { len = 0; return pos; }
    if (n > (uint64_t)(end - pos)) { fail(ST_MALFORMED); len = 0; return pos; }
    const uint32_t s = pos; pos += (uint32_t)n; len = (uint32_t)n; return s;
  }
};

// utf8_u16 (strict UTF-8, UTF-16 length or -1) over global memory by aligned 16-byte chunks: a
// chunk of ASCII counts its bytes at once, any other chunk runs the decoder over its registers
YDEV int64_t gutf8_u16(const uint8_t* s, uint32_t n) {
  int64_t u16 = 0;
  uint32_t rem = 0, cp = 0, mn = 0;
  const uintptr_t a0 = (uintptr_t)s, a1 = a0 + n;
  for (uintptr_t b = a0 & ~(uintptr_t)15; b < a1; b += 16) {
    const uint4 v = *(const uint4*)b;
    const uint32_t lo = b < a0 ? (uint32_t)(a0 - b) : 0u, hi = a1 - b < 16 ? (uint32_t)(a1 - b) : 16u;   // bytes [lo, hi) are ours
    const uint64_t x0 = ((uint64_t)v.y << 32) | v.x, x1 = ((uint64_t)v.w << 32) | v.z;
    uint64_t m0 = 0x8080808080808080ull, m1 = 0x8080808080808080ull;
    if (lo) { if (lo >= 8) { m0 = 0; m1 &= ~0ull << (8u * (lo - 8)); } else m0 &= ~0ull << (8u * lo); }
    if (hi < 16) { if (hi <= 8) { m1 = 0; m0 &= hi == 8 ? ~0ull : ((1ull << (8u * hi)) - 1ull); } else m1 &= (1ull << (8u * (hi - 8))) - 1ull; }
    if (rem == 0 && (x0 & m0) == 0 && (x1 & m1) == 0) { u16 += hi - lo; continue; }
    for (uint32_t i = lo; i < hi; i++) {
      const uint32_t c = (uint32_t)((i < 8 ? x0 >> (8 * i) : x1 >> (8 * (i - 8))) & 0xFFu);
      if (rem == 0) {
        if (c < 0x80u) { u16++; continue; }
        if ((c & 0xE0u) == 0xC0u) { rem = 1; cp = c & 0x1Fu; mn = 0x80; }
        else if ((c & 0xF0u) == 0xE0u) { rem = 2; cp = c & 0x0Fu; mn = 0x800; }
        else if ((c & 0xF8u) == 0xF0u) { rem = 3; cp = c & 0x07u; mn = 0x10000; }
        else return -1;
      } else {
        if ((c & 0xC0u) != 0x80u) return -1;
        cp = (cp << 6) | (c & 0x3Fu);
        if (--rem == 0) {
          if (cp < mn || cp > 0x10FFFFu || (cp >= 0xD800u && cp <= 0xDFFFu)) return -1;
          u16 += cp >= 0x10000u ? 2 : 1;
        }
      }
    }
  }
  return rem ? -1 : u16;
}

// One U0 struct: validated as read_struct (Y@81141 readers) and accepted only
// if write_struct(off = 0) reproduces its bytes (canonical info byte, parentInfo 0/1, minimal
// varuints, canonical content).  Returns the clock length; kind: 0 GC, 1 Item; ok = false defers.
struct GStruct { uint64_t len; uint32_t kind; bool ok, patch; };   // patch: written back with info bit 0x20 cleared
template <class CUR = GCur>
YDEV GStruct big_struct(CUR& c, uint32_t flags) {
  GStruct R; R.len = 0; R.kind = 1; R.ok = false; R.patch = false;
  c.nm = 0;
  const uint32_t info = c.u8();
  if (c.err) return R;
  if (info == 10u) return R;                                       // Skip: filtered by the reader -> general path
  if ((info & 31u) == 0u) {                                        // GC
    R.kind = 0; R.len = c.vu();
    R.ok = !c.err && !c.nm && info == 0u;
    return R;
  }
  const uint32_t ref = info & 31u;
  const bool ho = (info & 0x80u) != 0, hr = (info & 0x40u) != 0;
  // bit 0x20 beside an origin: Item.write keeps an integrated map entry's parentSub bit, the lazy reader drops it (its
  // parentSub is read only without origins), so yjs's merge writes the same struct with the bit cleared
  if ((ho || hr) && (info & 0x20u)) R.patch = true;
  if (ho) { c.vu(); c.vu(); }
  if (hr) { c.vu(); c.vu(); }
  if (!ho && !hr) {
    const uint64_t pi = c.vu();
    if (pi == 1) { uint32_t l; const uint32_t s0 = c.buf(l); if (!c.err && gutf8_u16(c.gp() + s0, l) < 0) return R; }
    else if (pi == 0) { c.vu(); c.vu(); }
    else return R;                                                 // parentInfo re-encoded as 0
    if (info & 0x20u) { uint32_t l; const uint32_t s0 = c.buf(l); if (!c.err && gutf8_u16(c.gp() + s0, l) < 0) return R; }
  }
  if (c.err || c.nm) return R;
  bool nc = false;
  switch (ref) {
    case 1: R.len = c.vu(); break;                                 // ContentDeleted
    case 2: {                                                      // ContentJSON
      const uint64_t n = c.vu();
      for (uint64_t k = 0; k < n && !c.err; k++) {
        uint32_t l; const uint32_t s = c.buf(l); if (c.err) break;
        if (gutf8_u16(c.gp() + s, l) < 0) return R;
        const uint8_t* t = c.gp() + s;
        if (l == 9 && t[0] == 'u' && t[1] == 'n' && t[2] == 'd' && t[3] == 'e' && t[4] == 'f' && t[5] == 'i' && t[6] == 'n' && t[7] == 'e' && t[8] == 'd') continue;
        if (json_check_t<SM_DEPTH, SM_KEYS>(t, l, nc)) return R;
      }
      R.len = n; break;
    }
    case 3: { uint32_t l; c.buf(l); R.len = 1; break; }            // ContentBinary
    case 4: {                                                      // ContentString
      uint32_t l; const uint32_t s = c.buf(l); if (c.err) return R;
      const int64_t u = gutf8_u16(c.gp() + s, l);
      if (u < 0) return R;
      R.len = (uint64_t)u; break;
    }
    case 5: {                                                      // ContentEmbed
      uint32_t l; const uint32_t s = c.buf(l); if (c.err) return R;
      if (gutf8_u16(c.gp() + s, l) < 0 || json_check_t<SM_DEPTH, SM_KEYS>(c.gp() + s, l, nc)) return R;
      R.len = 1; break;
    }
    case 6: {                                                      // ContentFormat
      uint32_t l; uint32_t s = c.buf(l); if (c.err) return R;
      if (gutf8_u16(c.gp() + s, l) < 0) return R;
      s = c.buf(l); if (c.err) return R;
      if (gutf8_u16(c.gp() + s, l) < 0 || json_check_t<SM_DEPTH, SM_KEYS>(c.gp() + s, l, nc)) return R;
      R.len = 1; break;
    }
    case 7: {                                                      // ContentType
      const uint64_t tr = c.vu(); if (c.err || tr > 6) return R;
      if (tr == 3 || tr == 5) { uint32_t l; const uint32_t s = c.buf(l); if (c.err || gutf8_u16(c.gp() + s, l) < 0) return R; }
      R.len = 1; break;
    }
    case 8: {                                                      // ContentAny (e.g. XmlElement attributes)
      const uint64_t n = c.vu(); if (c.err || n == 0) return R;
      Cur q{c.gp(), c.pos, c.end, 0, 0};
      for (uint64_t k = 0; k < n && !q.err; k++) any_value_t<SM_DEPTH, SM_KEYS>(q, nc, flags);   // readAny + would writeAny reproduce it
      if (q.err) return R;
      c.pos = q.pos;
      R.len = n; break;
    }
    default: return R;                                             // Doc (validated by the general path), bad refs
  }
  R.ok = !c.err && !c.nm && !nc;
  return R;
}

// one Any value skipped over global memory (lib0 readAny's layout); false on an unknown tag or nesting
// deeper than MAX_DEPTH (the document then goes on to the general path).  Out of line: the chain follow's
// fallback parse only.
YDEV_NI bool gany_skip(GCur& c, uint64_t n) {
  uint32_t rem[SM_DEPTH + 1], obj[SM_DEPTH + 1];   // (deeper values: the general path)
  int d = 0; rem[0] = n > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)n; obj[0] = 0;
  while (!c.err) {
    if (rem[d] == 0) { if (d == 0) return true; d--; continue; }
    rem[d]--;
    if (obj[d]) { uint32_t kl; c.buf(kl); if (c.err) return false; }
    const uint32_t tag = c.u8();
    switch (tag) {
      case 127: case 126: case 121: case 120: break;
      case 125: { uint32_t r = c.u8(); while ((r & 128u) && !c.err) r = c.u8(); break; }
      case 124: if (c.end - c.pos < 4) c.fail(ST_MALFORMED); else c.pos += 4; break;
      case 123: case 122: if (c.end - c.pos < 8) c.fail(ST_MALFORMED); else c.pos += 8; break;
      case 119: case 116: { uint32_t l; c.buf(l); break; }
      case 117: case 118: {
        const uint64_t k = c.vu();
        if (c.err || d + 1 > SM_DEPTH || k > (uint64_t)(c.end - c.pos)) return false;
        d++; rem[d] = (uint32_t)k; obj[d] = tag == 118;
        break;
      }
      default: return false;
    }
  }
  return false;
}

// The origin / right-origin ids after an info byte (npair id pairs: 2 or 4 varuints) skipped from one 16-byte view of
// the stage and its terminator mask, instead of a dependent read per varuint: the cursor ends where the vu() calls
// would leave it, with nm set the same way (a varuint's last byte zero past its first).  Returns false (cursor
// untouched) when the ids do not end inside the view and the update or a varuint runs past 7 bytes: the vu() path.
#ifndef YGM_SKIP_MASK
#define YGM_SKIP_MASK 1
#endif
YDEV uint32_t top_bits8(uint64_t h) { return (uint32_t)((((h >> 7) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56); }
YDEV uint64_t zero_bytes8(uint64_t x) {   // 0x80 in each zero byte of x, exactly (no borrow between bytes)
  const uint64_t t = (x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full;
  return ~(t | x | 0x7F7F7F7F7F7F7F7Full);
}
YDEV bool lcur_skip_ids(LCur& c, uint32_t npair) {
  if (c.pos >= c.end) return false;
  uint64_t lo, hi;
  c.w16(c.pos, lo, hi);
  const uint32_t T = top_bits8(~lo & 0x8080808080808080ull) | (top_bits8(~hi & 0x8080808080808080ull) << 8);
  const uint32_t Z = top_bits8(zero_bytes8(lo)) | (top_bits8(zero_bytes8(hi)) << 8);
  uint32_t t = T;
  const uint32_t e1 = (uint32_t)__builtin_ctz(t | 0x80000000u); t &= t - 1u;
  const uint32_t e2 = (uint32_t)__builtin_ctz(t | 0x80000000u); t &= t - 1u;
  const uint32_t e3 = (uint32_t)__builtin_ctz(t | 0x80000000u); t &= t - 1u;
  const uint32_t e4 = (uint32_t)__builtin_ctz(t | 0x80000000u);
  const uint32_t e = npair == 2u ? e4 : e2;
  const bool lens = e1 < 7u && e2 - e1 <= 7u && (npair != 2u || (e3 - e2 <= 7u && e4 - e3 <= 7u));
  if (!(e < 16u && lens && c.pos + e < c.end)) return false;
  if (Z & ~(T << 1) & ~1u & ((2u << e) - 1u)) c.nm = 1;
  c.pos += e + 1u;
  return true;
}

// Skip-only parse of one U0 struct (the sequential part of the walk): the bytes it spans and its
// kind (0 GC, 1 Item); validation and lengths come later, in parallel (big_struct).  false: a
// Skip, Any / Doc content or an unknown ref -- the document goes on to the general path.
// cv (the scan): GC's / ContentDeleted's length, or ContentString's bytes as start << 32 | length
template <bool ANY = false, class CUR = GCur>   // ANY: any ContentAny (the out-of-line fallback parse); else scalar values only
YDEV bool big_skip(CUR& c, uint32_t& kind, uint64_t jcap = ~0ull, uint64_t* cv = nullptr) {   // jcap: most ContentJSON entries taken
  const uint32_t info = c.u8();
  kind = 1;
  if (c.err || info == 10u) return false;
  if ((info & 31u) == 0u) { kind = 0; const uint64_t n = c.vu(); if (cv) *cv = n; return !c.err; }
  uint32_t l;
  bool skipped = false;
#if YGM_SKIP_MASK
  if constexpr (std::is_same<CUR, LCur>::value) skipped = (info & 0xC0u) == 0u || lcur_skip_ids(c, ((info >> 7) & 1u) + ((info >> 6) & 1u));
#endif
  if (!skipped) {
    if (info & 0x80u) { c.vu(); c.vu(); }
    if (info & 0x40u) { c.vu(); c.vu(); }
  }
  if ((info & 0xC0u) == 0u) {
    const uint64_t pi = c.vu();
    if (pi == 1) c.buf(l); else { c.vu(); c.vu(); }
    if (info & 0x20u) c.buf(l);
  }
  switch (info & 31u) {
    case 1: { const uint64_t n = c.vu(); if (cv) *cv = n; break; }
    case 2: { const uint64_t n = c.vu(); if (n > jcap) return false; for (uint64_t k = 0; k < n && !c.err; k++) c.buf(l); break; }
    case 4: { const uint32_t s = c.buf(l); if (cv) *cv = ((uint64_t)s << 32) | l; break; }
    case 3: case 5: c.buf(l); break;
    case 6: c.buf(l); c.buf(l); break;
    case 7: { const uint64_t tr = c.vu(); if (tr == 3 || tr == 5) c.buf(l); break; }
    case 8: {
      const uint64_t n = c.vu();
      if (c.err) return false;
      if constexpr (ANY) { if (!gany_skip(c, n)) return false; break; }
      if (n > jcap) return false;
      for (uint64_t k = 0; k < n && !c.err; k++) {   // the speculative parse takes scalar values only (attributes)
        const uint32_t tag = c.u8();
        if (tag == 119u || tag == 116u) c.buf(l);
        else if (tag == 125u) { uint32_t r = c.u8(); while ((r & 128u) && !c.err) r = c.u8(); }
        else if (tag == 124u) c.pos += 4;
        else if (tag == 123u || tag == 122u) c.pos += 8;
        else if (tag < 120u) return false;   // (120, 121, 126, 127: no payload; arrays / objects: the fallback parse)
        if (c.pos > c.end) c.fail(ST_MALFORMED);
      }
      break;
    }
    default: return false;
  }
  return !c.err;
}

// U0 block table entry (global scratch)
struct BigBlk {
  uint64_t client, clock0, clock1;   // clock range [clock0, clock1)
  uint32_t b0, b1;                   // struct bytes [b0, b1) of U0
  uint32_t nst;
  uint32_t s0;                       // index of the block's first struct record (walk scratch)
  uint8_t first_gc, last_gc;
  uint8_t hcanon;                    // block header varuints minimal: U0 bytes [h0, b1) are the block as written
  uint8_t pad;
  uint32_t h0;                       // block header start in U0
};
// one U0 struct record (walk scratch): its bytes [start, end), then its clock length once validated
struct BigRec { uint32_t start, end, len; };
// log piece (LDS): one struct of a log update
struct BigPiece {
  uint64_t key;                      // (~client) << 32 | clock: ascending = client descending, clock ascending
  uint64_t src;                      // arena offset of the struct's bytes
  uint32_t len, nbg;                 // clock length; byte length | GC << 31
  uint32_t gi;                       // the parallel emit's plan: the piece's client group
  uint32_t pre;                      // ... and the inclusive prefix of the pieces' output bytes (Skip + struct)
  YDEV uint32_t nb() const { return nbg & 0x7FFFFFFFu; }
  YDEV bool gc() const { return (nbg >> 31) != 0; }
};
// one client group of the parallel emit's plan (the log pieces of one client and U0's block of it, if any)
struct BigGrp {
  uint32_t q0, qend, uslot;          // pieces [q0, qend); the U0 block goes before piece uslot (qend: after all)
  uint32_t hdr;                      // header bytes
  uint32_t flags;                    // 1: U0 has a block of the client (touched), 2: its first struct GC, 4: its last
  uint32_t nst, clock0, clock1, b0, b1;   // the U0 block: struct count, clock range, struct bytes
  uint32_t h0ins;                    // U0 position the group goes to: its block's header (touched) or the next block's
  uint32_t cnt, first, gapu;         // output struct count, first clock, Skip before the U0 block
  uint32_t upos;                     // offset of the U0 block's struct bytes within the group's output
  uint32_t rel;                      // offset of the group's output within the structs part (after the block count)
};
// log delete range: key as BigPiece.  The delete-set splice (big_ds_plan) annotates it against U0's entry of its client:
// ent (the first entry at or after its client; bit 31 set: U0's delete set lacks the client), U0 ranges [a, b1) it
// touches (overlap or adjacency),
// its span with them [s, e), and the byte offsets (from U0's delete set start) of U0 range a and range b1
struct BigRange { uint64_t key; uint32_t len, ent, a, b1, s, e, pa, pb; };

// U0 tile (LDS): CH positions of U0 from the tile origin (plus 64 bytes of overlap, so a block header starting
// among them ends inside, and 16 for the alignment shift), the snapshot scan's struct ends of those positions (nx:
// end - tile origin, bit 15 = GC; 0 = no parse) and jump tables: jp[k][i] is the struct start 2^(k+1) structs after
// position i (built from nx by doubling), BJ_NONE when the chain breaks (a position without an end) or passes the
// tile's CH positions on the way: the chain follow takes up to 64 structs of a block per step, lane j composing the
// tables along the bits of j.
constexpr int BJ_LV = 5;
constexpr uint32_t BJ_NONE = 0xFFFFu;
template <uint32_t CH>
struct BigTileT {
  uint4 b[(CH + 64 + 16) / 16];
  uint16_t nx[CH];
  uint16_t jp[BJ_LV][CH];
};
template <int MAXS, int MAXD>
struct BigLdsT {
  BigPiece pc[MAXS];
  BigRange rg[MAXD];
  uint32_t npc, nrg, bad, patch;   // patch: U0 holds structs whose info byte loses bit 0x20 (the scan's bitmap marks them)
};

}  // namespace ygm
