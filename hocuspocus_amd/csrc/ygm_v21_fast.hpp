// ygm_v21_fast.hpp -- update V2 -> V1 (UpdateDecoderV2's reads written as V1 bytes) for the
// shapes text logs produce, with every column decoder in registers.
//
// The general transcoder (ygm_v2.hpp v21) keeps its nine column decoders and the rest cursor in one Dec2 object
// that lives in scratch memory (1.2 KB per lane, one wave per SIMD).  Here an update's bytes are staged (LDS on the
// device, <= 128 bytes per lane) and decoded by named register decoders -- lib0 0.2.42 UintOptRle / IntDiffOptRle /
// Rle and the StringDecoder, the same reads as ygm_v2.hpp uo_read / id_read / rle_read / rd_string -- for updates
// whose every read stays inside its column: a read past a column's end (JavaScript's `undefined` arithmetic), a
// string that is not ASCII, content other than Deleted / String, values >= 2^32, the public conversion's normal-form
// checks: the update takes the general transcoder.  The tests compare both paths byte for byte.
#pragma once
#include "ygm_v2.hpp"

namespace ygm {
namespace v21f {

constexpr uint32_t F21_MAX = 128;   // bytes per update (a longer update takes the general path)

// a column (or the rest) of the staged update: bytes [pos, end) of the buffer
struct BCol { uint32_t pos, end; };

template <class P>
struct Src {
  P b;   // the update's staged bytes
  YDEV uint32_t at(uint32_t i) const { return (uint32_t)b[i]; }
};

// readVarUint inside the column (< 2^32, <= 5 bytes); ok cleared past the column or on a longer value
template <class S>
YDEV uint32_t b_vu(const S& s, BCol& c, bool& ok) {
  uint32_t v = 0;
#pragma unroll 1
  for (uint32_t k = 0; k < 5u; k++) {
    if (c.pos >= c.end) { ok = false; return 0; }
    const uint32_t x = s.at(c.pos++);
    v |= (x & 127u) << (7u * k);
    if (x < 128u) { if (k == 4u && (x & 0x70u)) ok = false; return v; }
  }
  ok = false;
  return 0;
}
// readVarInt (magnitude < 2^32): the magnitude, its sign at bit 32 (no second by-reference flag: two flags reaching one
// inlined store would merge into a pointer select, and both would move to scratch memory)
template <class S>
YDEV uint64_t b_vi(const S& s, BCol& c, bool& ok) {
  if (c.pos >= c.end) { ok = false; return 0; }
  uint32_t x = s.at(c.pos++);
  uint32_t v = x & 63u;
  const uint64_t sg = (uint64_t)((x >> 6) & 1u) << 32;
  if (!(x & 128u)) return v | sg;
#pragma unroll 1
  for (uint32_t k = 0; k < 4u; k++) {
    if (c.pos >= c.end) { ok = false; return 0; }
    x = s.at(c.pos++);
    v |= (x & 127u) << (6u + 7u * k);
    if (x < 128u) { if (k == 3u && (x & 0x60u)) ok = false; return v | sg; }   // (6 + 21 + 5 bits: < 2^32)
  }
  ok = false;
  return 0;
}
// UintOptRleDecoder (uo_read)
struct BUo { BCol c; uint32_t count, s; };
template <class S>
YDEV uint32_t b_uo(const S& s, BUo& d, bool& ok) {
  if (d.count == 0u) {
    const uint64_t r = b_vi(s, d.c, ok);
    d.s = (uint32_t)r; d.count = 1u;
    if (r >> 32) { const uint32_t k = b_vu(s, d.c, ok); d.count = k + 2u; ok = ok && k < 0x7FFFFFF0u; }
  }
  d.count--;
  return d.s;
}
// IntDiffOptRleDecoder (id_read); the value must stay in [0, 2^32) (a clock)
struct BId { BCol c; uint32_t count; int64_t s, diff; };
template <class S>
YDEV uint32_t b_id(const S& s, BId& d, bool& ok) {
  if (d.count == 0u) {
    const uint64_t r = b_vi(s, d.c, ok);
    const uint32_t m = (uint32_t)r;
    const int32_t t = (int32_t)((r >> 32) ? 0u - m : m);
    d.diff = t >> 1; d.count = 1u;
    if (t & 1) { const uint32_t k = b_vu(s, d.c, ok); d.count = k + 2u; ok = ok && k < 0x7FFFFFF0u; }
  }
  d.s += d.diff;
  d.count--;
  ok = ok && d.s >= 0 && d.s <= 0xFFFFFFFFll;
  return (uint32_t)d.s;
}
// RleDecoder (rle_read) of bytes; an exhausted column (JS: undefined) is off the fast path
struct BRle { BCol c; int64_t count; uint32_t s; };
template <class S>
YDEV uint32_t b_rle(const S& s, BRle& d, bool& ok) {
  if (d.count == 0) {
    if (d.c.pos >= d.c.end) { ok = false; return 0; }
    d.s = s.at(d.c.pos++);
    if (d.c.pos != d.c.end) { const uint32_t k = b_vu(s, d.c, ok); d.count = (int64_t)k + 1; }
    else d.count = -1;   // (hasContent false: the value repeats)
  }
  d.count--;
  return d.s;
}

// output sink: counts, and stores when o != nullptr (bytes, varuints)
template <class Q>
struct BOut {
  Q o; uint32_t n;
  YDEV void b(uint32_t v) { if (o) o[n] = (uint8_t)v; n++; }
  YDEV void vu(uint32_t v) {
    if (!o) { n += 1u + (v > 0x7Fu) + (v > 0x3FFFu) + (v > 0x1FFFFFu) + (v > 0xFFFFFFFu); return; }
    while (v > 127u) { b(0x80u | (v & 127u)); v >>= 7; }
    b(v);
  }
};

// StringDecoder.read (rd_string): the next UTF-16 length (= bytes: ASCII) of the joined string -> varString
template <class S, class Q>
YDEV void b_str(const S& s, BUo& lens, uint32_t& sb, uint32_t sn, BOut<Q>& o, bool& ok) {
  const uint32_t want = b_uo(s, lens, ok);
  ok = ok && want <= sn - sb;
  if (!ok) return;
  o.vu(want);
  for (uint32_t i = 0; i < want; i++) o.b(s.at(sb + i));
  sb += want;
}

// V2 -> V1 of the staged update [0, n).  mode: 0 or v2::M_STRUCTS_ONLY (the public conversion, M_EXPORT, with its
// normal-form checks is the general path's).  Returns false off the fast path (o may hold a partial output then).
template <class S, class Q>
YDEV bool v21_fast(const S& s, uint32_t n, uint32_t mode, BOut<Q>& o) {
  if (n > F21_MAX || (mode & v2::M_EXPORT)) return false;
  bool ok = true;
  BCol rest{0u, n};
  (void)b_vu(s, rest, ok);   // (the leading varuint)
  BCol cols[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t l = b_vu(s, rest, ok);
    cols[i] = BCol{rest.pos, rest.pos + l};
    ok = ok && l <= n - (rest.pos < n ? rest.pos : n);
    rest.pos += l;
  }
  if (!ok) return false;
  // the string column: varString of every string joined (ASCII only here), then the UTF-16 lengths
  BCol sc = cols[5];
  const uint32_t sl = b_vu(s, sc, ok);
  const uint32_t s0 = sc.pos;
  ok = ok && sl <= sc.end - (sc.pos < sc.end ? sc.pos : sc.end);
  for (uint32_t i = 0; i < sl && ok; i++) ok = s.at(s0 + i) < 0x80u;
  if (!ok) return false;
  sc.pos += sl;
  uint32_t sb = s0;
  const uint32_t sn = s0 + sl;
  BUo lens{sc, 0u, 0u}, cl{cols[1], 0u, 0u}, ln{cols[8], 0u, 0u};
  BId lc{cols[2], 0u, 0, 0}, rc{cols[3], 0u, 0, 0};
  BRle info{cols[4], 0, 0u}, pi{cols[6], 0, 0u};
  const uint32_t nb = b_vu(s, rest, ok);
  o.vu(nb);
#pragma unroll 1
  for (uint32_t b = 0; b < nb && ok; b++) {
    const uint32_t ns = b_vu(s, rest, ok), client = b_uo(s, cl, ok), clock = b_vu(s, rest, ok);
    o.vu(ns); o.vu(client); o.vu(clock);
#pragma unroll 1
    for (uint32_t st = 0; st < ns && ok; st++) {
      const uint32_t inf = b_rle(s, info, ok);
      if (!ok) break;
      if (inf == 10u) { o.b(10u); o.vu(b_vu(s, rest, ok)); continue; }                // Skip
      if ((inf & 31u) == 0u) { o.b(0u); o.vu(b_uo(s, ln, ok)); continue; }             // GC
      const uint32_t ref = inf & 31u;
      ok = ok && (ref == 1u || ref == 4u);
      if (!ok) break;
      o.b(inf);
      if (inf & 0x80u) { o.vu(b_uo(s, cl, ok)); o.vu(b_id(s, lc, ok)); }
      if (inf & 0x40u) { o.vu(b_uo(s, cl, ok)); o.vu(b_id(s, rc, ok)); }
      if ((inf & 0xC0u) == 0u) {
        const uint32_t p = b_rle(s, pi, ok);
        if (p == 1u) { o.b(1u); b_str(s, lens, sb, sn, o, ok); }
        else { o.b(0u); o.vu(b_uo(s, cl, ok)); o.vu(b_id(s, lc, ok)); }
        if (inf & 0x20u) b_str(s, lens, sb, sn, o, ok);
      }
      if (ref == 1u) o.vu(b_uo(s, ln, ok));   // ContentDeleted
      else b_str(s, lens, sb, sn, o, ok);                             // ContentString
    }
  }
  if (!ok) return false;
  if (mode & v2::M_STRUCTS_ONLY) { o.b(0u); return true; }
  // delete set: V2 (clock - previous end, len - 1) -> V1 (clock, len)
  const uint32_t nd = b_vu(s, rest, ok);
  o.vu(nd);
#pragma unroll 1
  for (uint32_t i = 0; i < nd && ok; i++) {
    const uint32_t client = b_vu(s, rest, ok), nr = b_vu(s, rest, ok);
    o.vu(client); o.vu(nr);
    uint64_t cur = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < nr && ok; k++) {
      cur += b_vu(s, rest, ok);
      const uint64_t clock = cur, len = (uint64_t)b_vu(s, rest, ok) + 1u;
      cur += len;
      ok = ok && cur <= 0xFFFFFFFFull;
      o.vu((uint32_t)clock); o.vu((uint32_t)len);
    }
  }
  return ok;
}

}  // namespace v21f
}  // namespace ygm
