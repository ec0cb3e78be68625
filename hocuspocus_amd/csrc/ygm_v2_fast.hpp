// ygm_v2_fast.hpp -- V1 -> update V2 (UpdateEncoderV2 through yjs 13.6 convertUpdateFormat)
// for the shapes a merge / diff of text logs produces, with every encoder state in registers.
//
// The general transcoder (ygm_v2.hpp v12_body) keeps its eleven column writers in an array and its reads in a
// byte cursor: on the GPU that state lives in scratch and a C2 document costs ~30 us per struct.  Here one
// document's V1 bytes are staged (LDS on the device), structs are decoded from a 40-byte register window by
// its terminator mask (bit i: byte i has its top bit clear), and each column is a named register cursor.  Two
// passes over the same code: W = false counts the column lengths, W = true writes the columns at the offsets
// of the V2 layout (toUint8Array: 0, keyClock, client, leftClock, rightClock, info, string(+lens), parentInfo,
// typeRef, len, rest).
//
// Taken: client blocks (non-empty, consecutive clients distinct), GC, Skip, Items with origin and/or right
// origin or with a parent (parentInfo 1: a root-type key; 0: a parent id) and an optional parentSub, content
// ContentDeleted / ContentString (ASCII: UTF-16 length = bytes), the delete set (ranges in clock order per
// client), values < 2^32.  Anything else returns false and the document takes v12_body; the encoders below
// follow the same lib0 0.2.42 rules (rle_w / uo_w / id_w and their flushes, ygm_v2.hpp) -- the tests compare
// both paths byte for byte.
#pragma once
#include "ygm_v2.hpp"

namespace ygm {
namespace v2f {

constexpr uint32_t F_IN = 7168;    // staged V1 bytes (a document past this takes the general path)
constexpr uint32_t F_OUT = 6144;   // V2 bytes assembled per document

// lib0 encoder states (ygm_v2.hpp RleE / UoE / IdE with 32-bit values: the fast path takes values < 2^32)
struct FRle { uint32_t count; int32_t s; };
struct FUo { uint32_t count; uint32_t s; };
struct FId { uint32_t count; int64_t s, diff; };

// column cursors: byte count and (write pass) base offset in the output
struct FCol { uint32_t base, n; };
struct FEnc {
  FCol cl, lc, rc, info, str, lens, pi, ln, rest;
  FUo ucl, uln, ulens;
  FId ilc, irc;
  FRle rinfo, rpi;
};

template <class P>
YDEV uint32_t f_ld32(P p, uint32_t i) {   // dword i of a 4-byte aligned byte buffer
#ifdef YGM_HOST_BUILD
  uint32_t v; memcpy(&v, (const uint8_t*)p + 4u * i, 4); return v;
#else
  return ((const __attribute__((address_space(3))) uint32_t*)p)[i];
#endif
}
YDEV uint32_t f_align(uint32_t hi, uint32_t lo, uint32_t s) {   // bytes s.. of (hi:lo), s < 4
#ifdef YGM_HOST_BUILD
  return s ? (lo >> (8u * s)) | (hi << (32u - 8u * s)) : lo;
#else
  return __builtin_amdgcn_alignbyte(hi, lo, s);
#endif
}

// value of the <= 5-byte varuint whose first 4 bytes are x and 5th byte is y (n bytes)
YDEV uint32_t f_pext(uint32_t x, uint32_t y, uint32_t n) {
  x &= n >= 4u ? 0xFFFFFFFFu : ((1u << (8u * n)) - 1u);
  x &= 0x7f7f7f7fu;
  x = ((x >> 1) & 0x3f803f80u) | (x & 0x007f007fu);
  x = ((x >> 2) & 0x0fffc000u) | (x & 0x00003fffu);
  return x | (n >= 5u ? (y & 0x7Fu) << 28 : 0u);
}

// The staged input: bytes (4-byte aligned buffer, readable 64 bytes past the update) and its terminator masks
// (word k, bit i: byte 64 k + i has its top bit clear), built once per document by the whole wave.
template <class P, class M>
struct FSrc {
  P in; M m;
  YDEV uint32_t w32(uint32_t i) const { return f_ld32(in, i); }
  YDEV uint32_t byte(uint32_t p) const { return (w32(p >> 2) >> (8u * (p & 3u))) & 0xFFu; }
  YDEV uint64_t mask(uint32_t p) const {   // bit i: byte p + i ends a varuint
    const uint32_t k = p >> 6, s = p & 63u;
    const uint64_t lo = m[k], hi = m[k + 1u];
    return s ? (lo >> s) | (hi << (64u - s)) : lo;
  }
  YDEV void at5(uint32_t p, uint32_t& x, uint32_t& y) const {   // bytes p .. p + 4
    const uint32_t a = p >> 2, s = p & 3u;
    const uint32_t w0 = w32(a), w1 = w32(a + 1u);
    x = f_align(w1, w0, s);
    y = (w1 >> (8u * s)) & 0xFFu;
  }
};

// the reader: position p in the staged input (the update is [p0, n)); ok cleared on anything off the fast path
struct FRd {
  uint32_t p, n;
  bool ok;
};
// the varuint at q ending at byte e (both absolute, e >= q): its value; ok cleared past 5 bytes / 2^32 / n
template <class S>
YDEV uint32_t f_vat(const S& src, FRd& r, uint32_t q, uint32_t e) {
  uint32_t x, y;
  src.at5(q, x, y);
  const uint32_t nb = e - q + 1u;
  r.ok = r.ok && nb <= 5u && !(nb == 5u && (y & 0x70u)) && e < r.n;
  return f_pext(x, y, nb > 5u ? 5u : nb);
}
// next varuint (< 2^32): its mask and bytes are read together (one LDS round trip)
template <class S>
YDEV uint32_t f_vu(const S& src, FRd& r) {
  const uint64_t t = src.mask(r.p);
  const uint32_t e = r.p + (t ? (uint32_t)__builtin_ctzll(t) : 64u);
  const uint32_t v = f_vat(src, r, r.p, e);
  r.p = e + 1u;
  return v;
}
template <class S>
YDEV uint32_t f_u8(const S& src, FRd& r) {
  r.ok = r.ok && r.p < r.n;
  return src.byte(r.p++);
}

// ---- column writers (W: store; always count)
template <bool W, class Q>
YDEV void f_b(Q out, FCol& c, uint32_t v) {
  if (W && out) out[c.base + c.n] = (uint8_t)v;   // (out == nullptr: a count pass through the same code)
  c.n++;
}
template <bool W, class Q>
YDEV void f_vuw(Q out, FCol& c, uint32_t v) {
  while (v > 127u) { f_b<W>(out, c, 0x80u | (v & 127u)); v >>= 7; }
  f_b<W>(out, c, v);
}
template <bool W, class Q>
YDEV void f_vi(Q out, FCol& c, uint32_t m, bool neg) {   // lib0 writeVarInt of a magnitude < 2^32 (any_vi)
  f_b<W>(out, c, (m > 63u ? 0x80u : 0u) | (neg ? 0x40u : 0u) | (m & 63u));
  m >>= 6;
  while (m > 0u) { f_b<W>(out, c, (m > 127u ? 0x80u : 0u) | (m & 127u)); m >>= 7; }
}
template <bool W, class Q>
YDEV void f_rle(Q out, FCol& c, FRle& e, int32_t v) {
  if (e.s == v) { e.count++; return; }
  if (e.count > 0u) f_vuw<W>(out, c, e.count - 1u);
  e.count = 1; f_b<W>(out, c, (uint32_t)v); e.s = v;
}
template <bool W, class Q>
YDEV void f_uo_flush(Q out, FCol& c, const FUo& e) {
  if (e.count > 0u) { f_vi<W>(out, c, e.s, e.count != 1u); if (e.count > 1u) f_vuw<W>(out, c, e.count - 2u); }
}
template <bool W, class Q>
YDEV void f_uo(Q out, FCol& c, FUo& e, uint32_t v) {
  if (e.s == v) { e.count++; return; }
  f_uo_flush<W>(out, c, e);
  e.count = 1; e.s = v;
}
template <bool W, class Q>
YDEV void f_id_flush(Q out, FCol& c, const FId& e) {
  if (e.count > 0u) {
    const int32_t v = (int32_t)(((uint32_t)(uint64_t)e.diff << 1) | (e.count == 1u ? 0u : 1u));
    f_vi<W>(out, c, v < 0 ? 0u - (uint32_t)v : (uint32_t)v, v < 0);
    if (e.count > 1u) f_vuw<W>(out, c, e.count - 2u);
  }
}
template <bool W, class Q>
YDEV void f_id(Q out, FCol& c, FId& e, int64_t v) {
  if (e.diff == v - e.s) { e.s = v; e.count++; return; }
  f_id_flush<W>(out, c, e);
  e.count = 1; e.diff = v - e.s; e.s = v;
}
// ASCII check of the input bytes [s, s + len) from the terminator masks (ASCII <=> top bit clear)
template <class S>
YDEV bool f_ascii(const S& src, uint32_t s, uint32_t len) {
  for (uint32_t i = 0; i < len; i += 64u) {
    const uint32_t k = len - i < 64u ? len - i : 64u;
    const uint64_t want = k >= 64u ? ~0ull : ((1ull << k) - 1ull);
    if ((src.mask(s + i) & want) != want) return false;
  }
  return true;
}
// the string bytes [s, s + len) (ASCII, checked) to the string column, its length to lens
template <bool W, class S, class Q>
YDEV void f_put_str(const S& src, Q out, FEnc& k, uint32_t s, uint32_t len) {
  if (W && out)
    for (uint32_t i = 0; i < len; i++) out[k.str.base + k.str.n + i] = (uint8_t)src.byte(s + i);
  k.str.n += len;
  f_uo<W>(out, k.lens, k.ulens, len);
}
// a varString at the reader (ASCII only)
template <bool W, class S, class Q>
YDEV void f_str(const S& src, Q out, FRd& r, FEnc& k) {
  const uint32_t len = f_vu(src, r);
  const uint32_t s = r.p;
  r.ok = r.ok && len <= r.n - (s < r.n ? s : r.n) && f_ascii(src, s, len);
  if (!r.ok) return;
  f_put_str<W>(src, out, k, s, len);
  r.p = s + len;
}

// One pass over the V1 update [p0, n) of the staged input.  Returns false off the fast path (the caller takes
// v12_body).  An Item with origin(s) is decoded from ONE terminator-mask window read beside its info byte: the
// ends of its origin varuints and of its content length are the next set bits, so every field value is read in
// one more round trip (no byte-serial walk).
template <bool W, class S, class Q>
YDEV bool f_run(const S& src, uint32_t p0, uint32_t n, Q out, FEnc& k) {
  FRd r{p0, n, true};
  k.ucl = FUo{0, 0}; k.uln = FUo{0, 0}; k.ulens = FUo{0, 0};
  k.ilc = FId{0, 0, 0}; k.irc = FId{0, 0, 0};
  k.rinfo = FRle{0, -1}; k.rpi = FRle{0, -1};
  k.cl.n = k.lc.n = k.rc.n = k.info.n = k.str.n = k.lens.n = k.pi.n = k.ln.n = k.rest.n = 0;
  const uint32_t nb = f_vu(src, r);
  f_vuw<W>(out, k.rest, nb);
  uint32_t prev = 0; bool have_prev = false;
  for (uint32_t b = 0; b < nb && r.ok; b++) {
    const uint32_t ns = f_vu(src, r), client = f_vu(src, r), clock = f_vu(src, r);
    r.ok = r.ok && ns != 0u && !(have_prev && client == prev);   // lazy-writer normal (else ENONCANON: v12_body decides)
    prev = client; have_prev = true;
    if (!r.ok) break;
    f_uo<W>(out, k.cl, k.ucl, client); f_vuw<W>(out, k.rest, ns); f_vuw<W>(out, k.rest, clock);
    for (uint32_t st = 0; st < ns && r.ok; st++) {
      const uint32_t p = r.p;
      r.ok = r.ok && p < r.n;
      const uint32_t info = src.byte(p);
      const uint64_t m = src.mask(p + 1u);          // (independent of the info byte: read together)
      const uint32_t ref = info & 31u;
      const bool ho = (info & 0x80u) != 0u, hr = (info & 0x40u) != 0u;
      if ((ho || hr) && (ref == 1u || ref == 4u) && !(info & 0x20u)) {
        // origin ids (2 or 4 varuints) and the content length: the next 3 or 5 terminators after the info byte
        uint64_t t = m;
        uint32_t e[5];
#pragma unroll
        for (int j = 0; j < 5; j++) { e[j] = t ? (uint32_t)__builtin_ctzll(t) : 64u; t &= t - 1ull; }
        const uint32_t nv = (ho && hr) ? 5u : 3u;
        const uint32_t el = nv == 5u ? e[4] : e[2];   // the content length's terminator
        if (el < 64u) {
          const uint32_t q = p + 1u;
          const uint32_t v0 = f_vat(src, r, q, q + e[0]), v1 = f_vat(src, r, q + e[0] + 1u, q + e[1]);
          const uint32_t v2 = f_vat(src, r, q + e[1] + 1u, q + e[2]);
          uint32_t v3 = 0, v4 = 0;
          if (nv == 5u) { v3 = f_vat(src, r, q + e[2] + 1u, q + e[3]); v4 = f_vat(src, r, q + e[3] + 1u, q + e[4]); }
          const uint32_t len = nv == 5u ? v4 : v2;
          const uint32_t cs = q + el + 1u;               // after the content length
          uint32_t next = cs;
          if (ref == 4u) {
            next = cs + len;
            r.ok = r.ok && len <= r.n - (cs < r.n ? cs : r.n) &&
                   (el + 1u + len < 64u ? ((~m >> (el + 1u)) & (len >= 64u ? ~0ull : ((1ull << len) - 1ull))) == 0ull
                                         : f_ascii(src, cs, len));
          }
          if (!r.ok) break;
          f_rle<W>(out, k.info, k.rinfo, (int32_t)(ref | (ho ? 0x80u : 0u) | (hr ? 0x40u : 0u)));
          if (ho) { f_uo<W>(out, k.cl, k.ucl, v0); f_id<W>(out, k.lc, k.ilc, (int64_t)v1); }
          if (hr) {
            f_uo<W>(out, k.cl, k.ucl, ho ? v2 : v0); f_id<W>(out, k.rc, k.irc, (int64_t)(ho ? v3 : v1));
          }
          if (ref == 1u) f_uo<W>(out, k.ln, k.uln, len);   // ContentDeleted
          else f_put_str<W>(src, out, k, cs, len);         // ContentString
          r.p = next;
          continue;
        }
      }
      // everything else, field by field
      r.p = p + 1u;
      if (info == 10u) {   // Skip (read_struct's order: info 10 exactly, then any info with ref 0 is a GC)
        f_rle<W>(out, k.info, k.rinfo, 10);
        f_vuw<W>(out, k.rest, f_vu(src, r));
        continue;
      }
      if (ref == 0u) {   // GC
        f_rle<W>(out, k.info, k.rinfo, 0);
        f_uo<W>(out, k.ln, k.uln, f_vu(src, r));
        continue;
      }
      r.ok = r.ok && (ref == 1u || ref == 4u);
      if (!r.ok) break;
      const bool hs = !ho && !hr && (info & 0x20u);
      f_rle<W>(out, k.info, k.rinfo, (int32_t)(ref | (ho ? 0x80u : 0u) | (hr ? 0x40u : 0u) | (hs ? 0x20u : 0u)));
      if (ho) { const uint32_t oc = f_vu(src, r), ok = f_vu(src, r); f_uo<W>(out, k.cl, k.ucl, oc); f_id<W>(out, k.lc, k.ilc, (int64_t)ok); }
      if (hr) { const uint32_t rc = f_vu(src, r), rk = f_vu(src, r); f_uo<W>(out, k.cl, k.ucl, rc); f_id<W>(out, k.rc, k.irc, (int64_t)rk); }
      if (!ho && !hr) {
        const uint32_t pi = f_vu(src, r);
        r.ok = r.ok && pi <= 1u;
        if (!r.ok) break;
        if (pi == 1u) { f_rle<W>(out, k.pi, k.rpi, 1); f_str<W>(src, out, r, k); }
        else {
          f_rle<W>(out, k.pi, k.rpi, 0);
          const uint32_t pc = f_vu(src, r), pk = f_vu(src, r);
          f_uo<W>(out, k.cl, k.ucl, pc); f_id<W>(out, k.lc, k.ilc, (int64_t)pk);
        }
        if (hs) f_str<W>(src, out, r, k);
      }
      if (ref == 1u) f_uo<W>(out, k.ln, k.uln, f_vu(src, r));   // ContentDeleted
      else f_str<W>(src, out, r, k);                            // ContentString
    }
  }
  if (!r.ok) return false;
  // delete set: V1 (clock, len) -> V2 (clock - previous end, len - 1)
  const uint32_t nd = f_vu(src, r);
  f_vuw<W>(out, k.rest, nd);
  for (uint32_t i = 0; i < nd && r.ok; i++) {
    const uint32_t client = f_vu(src, r), nr = f_vu(src, r);
    f_vuw<W>(out, k.rest, client); f_vuw<W>(out, k.rest, nr);
    uint64_t cur = 0;
    for (uint32_t q = 0; q < nr && r.ok; q++) {
      const uint32_t clock = f_vu(src, r), len = f_vu(src, r);
      r.ok = r.ok && (uint64_t)clock >= cur && len != 0u;   // (a backward clock / zero length: v12_body's rules)
      if (!r.ok) break;
      f_vuw<W>(out, k.rest, (uint32_t)(clock - cur)); f_vuw<W>(out, k.rest, len - 1u);
      cur = (uint64_t)clock + len;
    }
  }
  if (!r.ok) return false;
  f_uo_flush<W>(out, k.cl, k.ucl); f_id_flush<W>(out, k.lc, k.ilc); f_id_flush<W>(out, k.rc, k.irc);
  f_uo_flush<W>(out, k.lens, k.ulens); f_uo_flush<W>(out, k.ln, k.uln);
  return true;
}

// terminator masks of the staged bytes [0, nbytes) (nbytes a multiple of 64): word k for bytes 64 k ..
template <class P>
YDEV uint64_t f_mask_word(P in, uint32_t k) {
  uint64_t H = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t v = f_ld32(in, 16u * k + (uint32_t)j);
#pragma unroll
    for (int b = 0; b < 4; b++) H |= (uint64_t)((v >> (8 * b + 7)) & 1u) << (4 * j + b);
  }
  return ~H;
}

YDEV uint32_t f_vlen(uint32_t v) { return 1u + (v > 0x7Fu) + (v > 0x3FFFu) + (v > 0x1FFFFFu) + (v > 0xFFFFFFFu); }
// V2 size from the counted columns (ygm_v2.hpp v2_total; keyClock and typeRef are empty here)
YDEV uint32_t f_total(const FEnc& k) {
  uint32_t t = 1u + 2u;   // version 0, empty keyClock, empty typeRef
  t += f_vlen(k.cl.n) + k.cl.n + f_vlen(k.lc.n) + k.lc.n + f_vlen(k.rc.n) + k.rc.n + f_vlen(k.info.n) + k.info.n;
  const uint32_t sc = f_vlen(k.str.n) + k.str.n + k.lens.n;
  t += f_vlen(sc) + sc;
  t += f_vlen(k.pi.n) + k.pi.n + f_vlen(k.ln.n) + k.ln.n;
  return t + k.rest.n;
}
// writes the V2 header (version and column lengths) and sets each column's base
template <class Q>
YDEV void f_layout(Q out, FEnc& k) {
  FCol h{0u, 0u};
  f_b<true>(out, h, 0u);
  f_vuw<true>(out, h, 0u);                                                    // keyClock
  f_vuw<true>(out, h, k.cl.n); k.cl.base = h.n; h.n += k.cl.n;
  f_vuw<true>(out, h, k.lc.n); k.lc.base = h.n; h.n += k.lc.n;
  f_vuw<true>(out, h, k.rc.n); k.rc.base = h.n; h.n += k.rc.n;
  f_vuw<true>(out, h, k.info.n); k.info.base = h.n; h.n += k.info.n;
  const uint32_t sc = f_vlen(k.str.n) + k.str.n + k.lens.n;
  f_vuw<true>(out, h, sc); f_vuw<true>(out, h, k.str.n);
  k.str.base = h.n; h.n += k.str.n;
  k.lens.base = h.n; h.n += k.lens.n;
  f_vuw<true>(out, h, k.pi.n); k.pi.base = h.n; h.n += k.pi.n;
  f_vuw<true>(out, h, 0u);                                                    // typeRef
  f_vuw<true>(out, h, k.ln.n); k.ln.base = h.n; h.n += k.ln.n;
  k.rest.base = h.n;
}

}  // namespace v2f
}  // namespace ygm
