// ygm_v2_fast.hpp -- V1 -> update V2 (UpdateEncoderV2 through yjs 13.6 convertUpdateFormat)
// for the shapes a merge / diff of text logs produces.
//
// The general transcoder (ygm_v2.hpp v12_body) is one lane per document with its eleven column writers in an
// array and a byte cursor over global memory: on the GPU that state lives in scratch, ~30 us per struct.  Here a
// document's V1 bytes are staged (LDS on the device) with their terminator masks (bit i: byte i has its top bit
// clear), an Item's fields are located from one mask window beside its info byte, and the V2 columns are encoded
// one per lane (f_col_run): the lanes of a document walk the same bytes and each feeds its column's values to one
// generic encoder (lib0 0.2.42 UintOptRle / IntDiffOptRle / Rle, the string bytes, the rest column's varuints --
// ygm_v2.hpp rle_w / uo_w / id_w and their flushes).  A count pass sizes the columns, the layout places them
// (toUint8Array: 0, keyClock, client, leftClock, rightClock, info, string(+lens), parentInfo, typeRef, len, rest),
// a write pass stores them.
//
// Taken: client blocks (non-empty, consecutive clients distinct), GC, Skip, Items with origin and/or right
// origin or with a parent (parentInfo 1: a root-type key; 0: a parent id) and an optional parentSub, content
// ContentDeleted / ContentString (ASCII: UTF-16 length = bytes), the delete set (ranges in clock order per
// client), values < 2^32.  Anything else returns false and the document takes v12_body; the tests compare both
// paths byte for byte (tests/test_v2_fast_host.py on the host build, tests/test_v2.py on the GPU).
#pragma once
#include "ygm_v2.hpp"

namespace ygm {
namespace v2f {

constexpr uint32_t F_IN = 7168;    // staged V1 bytes (a document past this takes the general path)
constexpr uint32_t F_OUT = 6144;   // V2 bytes assembled per document

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

// ---------------------------------------------------------------- one column per lane
// The nine V2 columns a text log produces are encoded side by side, one lane each: every lane walks the same V1
// bytes (the decode is the same instruction stream for all of them, LDS reads broadcast), picks its column's
// values of each struct (up to three, in the writer's order) and feeds them to one generic encoder whose mode is
// data: lib0's UintOptRle / IntDiffOptRle / Rle, the string bytes, or the raw varuints of the rest column.
enum : uint32_t { FC_CL = 0, FC_LC, FC_RC, FC_INFO, FC_LENS, FC_PI, FC_LN, FC_STR, FC_REST, FC_N };
enum : uint32_t { FM_UOR = 0, FM_IDOR, FM_RLE, FM_STR, FM_VU };
YDEV uint32_t f_mode(uint32_t col) {
  return col == FC_LC || col == FC_RC ? FM_IDOR : col == FC_INFO || col == FC_PI ? FM_RLE : col == FC_STR ? FM_STR
       : col == FC_REST ? FM_VU : FM_UOR;
}
struct FCS { uint32_t mode, n, count, cap; int64_t s, diff; };   // one column's encoder, byte count, store capacity
template <class Q>
YDEV void fc_b(Q out, uint32_t base, FCS& c, uint32_t v) {
  if (out && c.n < c.cap) out[base + c.n] = (uint8_t)v;   // (out == nullptr: a count pass; past cap: counted only,
  c.n++;                                                   //  the caller sees c.n > cap and refuses the document)
}
template <class Q>
YDEV void fc_vu(Q out, uint32_t base, FCS& c, uint32_t v) {
  if (!out) { c.n += 1u + (v > 0x7Fu) + (v > 0x3FFFu) + (v > 0x1FFFFFu) + (v > 0xFFFFFFFu); return; }   // count pass: no loop
  while (v > 127u) { fc_b(out, base, c, 0x80u | (v & 127u)); v >>= 7; }
  fc_b(out, base, c, v);
}
template <class Q>
YDEV void fc_vi(Q out, uint32_t base, FCS& c, uint32_t m, bool neg) {   // lib0 writeVarInt of a magnitude < 2^32
  if (!out) { c.n += 1u + (m > 0x3Fu) + (m > 0x1FFFu) + (m > 0xFFFFFu) + (m > 0x7FFFFFFu); return; }
  fc_b(out, base, c, (m > 63u ? 0x80u : 0u) | (neg ? 0x40u : 0u) | (m & 63u));
  m >>= 6;
  while (m > 0u) { fc_b(out, base, c, (m > 127u ? 0x80u : 0u) | (m & 127u)); m >>= 7; }
}
// the pending run of a UintOptRle / IntDiffOptRle column (uo_flush / id_flush)
template <class Q>
YDEV void fc_flush(Q out, uint32_t base, FCS& c) {
  if (c.count == 0u || c.mode > FM_IDOR) return;
  uint32_t mag; bool neg;
  if (c.mode == FM_UOR) { mag = (uint32_t)c.s; neg = c.count != 1u; }
  else {
    const int32_t v = (int32_t)(((uint32_t)(uint64_t)c.diff << 1) | (c.count == 1u ? 0u : 1u));
    neg = v < 0; mag = neg ? 0u - (uint32_t)v : (uint32_t)v;
  }
  fc_vi(out, base, c, mag, neg);
  if (c.count > 1u) fc_vu(out, base, c, c.count - 2u);
}
// one value into the column (FM_STR: the staged input bytes [off, off + v))
template <class S, class Q>
YDEV void fc_push(const S& src, Q out, uint32_t base, FCS& c, uint32_t v, uint32_t off) {
  if (c.mode == FM_VU) { fc_vu(out, base, c, v); return; }
  if (c.mode == FM_STR) {
    if (out) for (uint32_t i = 0; i < v && c.n + i < c.cap; i++) out[base + c.n + i] = (uint8_t)src.byte(off + i);
    c.n += v;
    return;
  }
  if (c.mode == FM_RLE) {   // rle_w
    if ((int64_t)v == c.s) { c.count++; return; }
    if (c.count > 0u) fc_vu(out, base, c, c.count - 1u);
    fc_b(out, base, c, v); c.s = (int64_t)v; c.count = 1u;
    return;
  }
  const bool id = c.mode == FM_IDOR;   // uo_w / id_w
  const int64_t key = id ? (int64_t)v - c.s : (int64_t)v, cur = id ? c.diff : c.s;
  if (key == cur) { c.count++; if (id) c.s = (int64_t)v; return; }
  fc_flush(out, base, c);
  c.count = 1u;
  if (id) c.diff = key;
  c.s = (int64_t)v;
}
// the up-to-three values (v, off) of one step for one column; bit j of pm: value j present
struct FCand { uint32_t v0, v1, v2, o0, o1, o2, pm; };
YDEV FCand fc_one(bool on, uint32_t v) { return FCand{v, 0, 0, 0, 0, 0, on ? 1u : 0u}; }
YDEV FCand fc_two(bool on, uint32_t v0, uint32_t v1) { return FCand{v0, v1, 0, 0, 0, 0, on ? 3u : 0u}; }

// Column `col` of the V2 encoding of the V1 update [p0, n) of the staged input: its bytes to out + base (out ==
// nullptr: counts c.n only).  Returns false off the fast path (every lane of a document sees the same bytes, so
// all of them return the same).  The walk is ONE loop whose body decodes one step of the update (its header, a
// block header, a struct, a delete-set header / client / range) and hands the column's values of that step to ONE
// inlined encoder: the kernel's code must stay small enough for the instruction cache (a walk with an encoder
// inlined at every value site ran ~20x slower, instruction-fetch bound).
enum : uint32_t { FP_DOC = 0, FP_BLK, FP_ST, FP_DSH, FP_DSC, FP_DSR, FP_DONE };
template <class S, class Q>
YDEV bool f_col_run(const S& src, uint32_t p0, uint32_t n, uint32_t col, Q out, uint32_t base, uint32_t cap, FCS& c) {
  c.mode = f_mode(col); c.n = 0; c.count = 0; c.cap = cap; c.s = c.mode == FM_RLE ? -1 : 0; c.diff = 0;
  FRd r{p0, n, true};
  const bool rest = col == FC_REST;
  uint32_t ph = FP_DOC, nb = 0, b = 0, ns = 0, st = 0, prev = 0, nd = 0, di = 0, nr = 0, q = 0;
  bool have_prev = false;
  uint64_t cur = 0;
#pragma unroll 1
  while (ph != FP_DONE && r.ok) {
    FCand k{0, 0, 0, 0, 0, 0, 0};
    if (ph == FP_DOC) {
      nb = f_vu(src, r); b = 0;
      k = fc_one(rest, nb);
      ph = nb ? FP_BLK : FP_DSH;
    } else if (ph == FP_BLK) {
      ns = f_vu(src, r); const uint32_t client = f_vu(src, r), clock = f_vu(src, r);
      r.ok = r.ok && ns != 0u && !(have_prev && client == prev);   // lazy-writer normal (else ENONCANON: v12_body decides)
      prev = client; have_prev = true; st = 0;
      k = FCand{col == FC_CL ? client : ns, clock, 0, 0, 0, 0, col == FC_CL ? 1u : rest ? 3u : 0u};
      ph = FP_ST;
    } else if (ph == FP_ST) {
      const uint32_t p = r.p;
      r.ok = r.ok && p < r.n;
      const uint32_t info = src.byte(p);
      const uint64_t m = src.mask(p + 1u);          // (independent of the info byte: read together)
      const uint32_t ref = info & 31u;
      const bool ho = (info & 0x80u) != 0u, hr = (info & 0x40u) != 0u;
      // the struct's fields (one decode for all columns)
      uint32_t code = 0, oc = 0, ok = 0, rc = 0, rk = 0, pi = 0, pc = 0, pk = 0, len = 0;
      uint32_t ko = 0, kl = 0, so = 0, sl = 0, co = 0;
      bool gc = false, skip = false, item = false, has_pid = false, has_key = false, hs = false;
      // an Item with origin ids (2 or 4 varuints) and a content length: the next 3 or 5 terminators after the
      // info byte locate every field, read in one more round trip
      uint64_t t = m;
      uint32_t e0, e1, e2, e3, e4;
      e0 = t ? (uint32_t)__builtin_ctzll(t) : 64u; t &= t - 1ull;
      e1 = t ? (uint32_t)__builtin_ctzll(t) : 64u; t &= t - 1ull;
      e2 = t ? (uint32_t)__builtin_ctzll(t) : 64u; t &= t - 1ull;
      e3 = t ? (uint32_t)__builtin_ctzll(t) : 64u; t &= t - 1ull;
      e4 = t ? (uint32_t)__builtin_ctzll(t) : 64u;
      const uint32_t el = (ho && hr) ? e4 : e2;     // the content length's terminator
      if ((ho || hr) && (ref == 1u || ref == 4u) && !(info & 0x20u) && el < 64u) {
        const uint32_t q1 = p + 1u;
        const uint32_t v0 = f_vat(src, r, q1, q1 + e0), v1 = f_vat(src, r, q1 + e0 + 1u, q1 + e1);
        const uint32_t v2 = f_vat(src, r, q1 + e1 + 1u, q1 + e2);
        const uint32_t v3 = (ho && hr) ? f_vat(src, r, q1 + e2 + 1u, q1 + e3) : 0u;
        const uint32_t v4 = (ho && hr) ? f_vat(src, r, q1 + e3 + 1u, q1 + e4) : 0u;
        len = (ho && hr) ? v4 : v2;
        co = q1 + el + 1u;                              // after the content length
        uint32_t next = co;
        if (ref == 4u) {
          next = co + len;
          r.ok = r.ok && len <= r.n - (co < r.n ? co : r.n) &&
                 (el + 1u + len < 64u ? ((~m >> (el + 1u)) & (len >= 64u ? ~0ull : ((1ull << len) - 1ull))) == 0ull
                                      : f_ascii(src, co, len));
        }
        item = true;
        code = ref | (ho ? 0x80u : 0u) | (hr ? 0x40u : 0u);
        oc = v0; ok = v1;
        rc = ho ? v2 : v0; rk = ho ? v3 : v1;
        r.p = next;
      } else {   // everything else, field by field
        r.p = p + 1u;
        if (info == 10u) { skip = true; code = 10u; len = f_vu(src, r); }   // Skip (info 10 exactly; then ref 0 is a GC)
        else if (ref == 0u) { gc = true; code = 0u; len = f_vu(src, r); }   // GC
        else {
          r.ok = r.ok && (ref == 1u || ref == 4u);
          item = true;
          hs = !ho && !hr && (info & 0x20u);
          code = ref | (ho ? 0x80u : 0u) | (hr ? 0x40u : 0u) | (hs ? 0x20u : 0u);
          if (ho) { oc = f_vu(src, r); ok = f_vu(src, r); }
          if (hr) { rc = f_vu(src, r); rk = f_vu(src, r); }
          if (!ho && !hr) {
            pi = f_vu(src, r);
            r.ok = r.ok && pi <= 1u;
            if (pi == 1u) {   // a root type's key
              has_key = true; kl = f_vu(src, r); ko = r.p;
              r.ok = r.ok && kl <= r.n - (ko < r.n ? ko : r.n) && f_ascii(src, ko, kl);
              r.p = ko + kl;
            } else { has_pid = true; pc = f_vu(src, r); pk = f_vu(src, r); }
            if (hs) {         // parentSub
              sl = f_vu(src, r); so = r.p;
              r.ok = r.ok && sl <= r.n - (so < r.n ? so : r.n) && f_ascii(src, so, sl);
              r.p = so + sl;
            }
          }
          len = f_vu(src, r);
          if (ref == 4u) {
            co = r.p;
            r.ok = r.ok && len <= r.n - (co < r.n ? co : r.n) && f_ascii(src, co, len);
            r.p = co + len;
          }
        }
      }
      const bool noo = item && !ho && !hr, str = item && ref == 4u, io = item && ho, ir = item && hr;   // (GC info bits are no origins)
      // this column's values of the struct, in v12_body's order (selects, not a branch per column)
      const uint32_t pcl = (io || ir ? 1u : 0u) | (io && ir ? 2u : 0u) | (has_pid ? 4u : 0u);
      const uint32_t pstr = (has_key ? 1u : 0u) | (hs ? 2u : 0u) | (str ? 4u : 0u);
      k.v0 = col == FC_CL ? (io ? oc : rc) : col == FC_LC ? ok : col == FC_RC ? rk : col == FC_INFO ? code
           : col == FC_LENS || col == FC_STR ? kl : col == FC_PI ? pi : len;
      k.v1 = col == FC_CL ? rc : col == FC_LC ? pk : sl;
      k.v2 = col == FC_CL ? pc : len;
      k.o0 = ko; k.o1 = so; k.o2 = co;
      k.pm = col == FC_CL ? pcl : col == FC_LC ? (io ? 1u : 0u) | (has_pid ? 2u : 0u) : col == FC_RC ? (ir ? 1u : 0u)
           : col == FC_INFO ? 1u : col == FC_LENS || col == FC_STR ? pstr : col == FC_PI ? (noo ? 1u : 0u)
           : col == FC_LN ? (gc || (item && ref == 1u) ? 1u : 0u) : (skip ? 1u : 0u);
      if (++st == ns) { b++; ph = b < nb ? FP_BLK : FP_DSH; }
    } else if (ph == FP_DSH) {   // delete set: V1 (clock, len) -> V2 (clock - previous end, len - 1), into the rest column
      nd = f_vu(src, r); di = 0;
      k = fc_one(rest, nd);
      ph = nd ? FP_DSC : FP_DONE;
    } else if (ph == FP_DSC) {
      const uint32_t client = f_vu(src, r);
      nr = f_vu(src, r); q = 0; cur = 0;
      k = fc_two(rest, client, nr);
      ph = nr ? FP_DSR : (++di < nd ? FP_DSC : FP_DONE);
    } else {   // FP_DSR
      const uint32_t clock = f_vu(src, r), len = f_vu(src, r);
      r.ok = r.ok && (uint64_t)clock >= cur && len != 0u;   // (a backward clock / zero length: v12_body's rules)
      k = fc_two(rest, (uint32_t)(clock - cur), len - 1u);
      cur = (uint64_t)clock + len;
      if (++q == nr) ph = ++di < nd ? FP_DSC : FP_DONE;
    }
    if (!r.ok) break;
    // the one encoder site: up to three values
#pragma unroll 1
    for (uint32_t j = 0; j < 3u; j++)
      if ((k.pm >> j) & 1u) fc_push(src, out, base, c, j == 0u ? k.v0 : j == 1u ? k.v1 : k.v2, j == 0u ? k.o0 : j == 1u ? k.o1 : k.o2);
  }
  if (!r.ok) return false;
  fc_flush(out, base, c);
  return true;
}
// V2 size and column bases (UpdateEncoderV2.toUint8Array layout) from the nine columns' byte counts L[FC_*];
// writes the header (version, column lengths) when out != nullptr.  base[FC_*] = each column's offset.
template <class Q>
YDEV uint32_t fc_layout(Q out, const uint32_t (&L)[FC_N], uint32_t (&base)[FC_N]) {
  FCS h{FM_VU, 0u, 0u, 0xFFFFFFFFu, 0, 0};
  fc_b(out, 0u, h, 0u);                                          // version
  fc_vu(out, 0u, h, 0u);                                         // keyClock (empty)
  const uint32_t pre[5] = {FC_CL, FC_LC, FC_RC, FC_INFO, FC_N};
#pragma unroll
  for (int q = 0; q < 4; q++) { fc_vu(out, 0u, h, L[pre[q]]); base[pre[q]] = h.n; h.n += L[pre[q]]; }
  uint32_t sv = L[FC_STR], vl = 1u;
  while (sv > 127u) { sv >>= 7; vl++; }
  fc_vu(out, 0u, h, vl + L[FC_STR] + L[FC_LENS]); fc_vu(out, 0u, h, L[FC_STR]);
  base[FC_STR] = h.n; h.n += L[FC_STR];
  base[FC_LENS] = h.n; h.n += L[FC_LENS];
  fc_vu(out, 0u, h, L[FC_PI]); base[FC_PI] = h.n; h.n += L[FC_PI];
  fc_vu(out, 0u, h, 0u);                                         // typeRef (empty)
  fc_vu(out, 0u, h, L[FC_LN]); base[FC_LN] = h.n; h.n += L[FC_LN];
  base[FC_REST] = h.n;
  return h.n + L[FC_REST];
}

}  // namespace v2f
}  // namespace ygm
