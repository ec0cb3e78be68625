// ygm_doc_lean.hpp -- encodeStateVectorFromUpdate / diffUpdate fast path: ONE LANE PER
// DOCUMENT, streaming the document through a 64-byte register window.
//
// The reconnect-sync shape: a merged document state (one update whose
// client blocks hold Items with String / Deleted / Type content, GC and Skip structs) and,
// for diff, a small state vector.  The former per-document kernel read global memory one
// byte at a time (one dependent load per byte); here each lane keeps bytes [cb, cb + 64) of
// its document in 16 VGPRs, refilled by aligned 16-byte loads as it advances, and decodes
// each struct from a normalised 32-byte view with the terminator mask of lean merge
// (ygm_merge_lean.hpp): varuint ends by ctz, no byte loop.
//
// Rules: R-SV (yjs Y@37728) and R-D (App. B.2, Y@40711), restated from
// sv_doc / DiffGen (ygm_seqdoc.hpp), which stay the exact reference for everything this
// kernel defers: content other than ASCII String / Deleted / Type, non-minimal varuints,
// values >= 2^32, repeated clients, delete sets that re-encode differently, > 16 state-vector
// entries.  Outputs go to per-document slots (no cross-document scan); the document header
// (a count known only at the end) is written right-aligned in front of the body.
#pragma once
#include "ygm_merge_lean.hpp"

namespace ygm {

constexpr int DL_SV_MAX = 16;   // state-vector entries held per lane (diff)

// Lane-private streaming window: W[0..15] = arena bytes [cb, cb + 64).
struct SWin {
  const uint8_t* base;   // arena
  uint64_t cb;           // absolute offset of W[0] (multiple of 16)
  uint64_t last;         // last loadable 16-byte chunk (arena tail padding >= 16)
  uint32_t W[16];
  YDEV u32x4 ld(uint64_t off) const { off = off < last ? off : last; return *(const u32x4*)(base + off); }
  YDEV void init(const uint8_t* b, uint64_t pos, uint64_t lastc) {
    base = b; last = lastc; cb = pos & ~15ull;
#pragma unroll
    for (int j = 0; j < 4; j++) { const u32x4 v = ld(cb + 16ull * j); W[4 * j] = v.x; W[4 * j + 1] = v.y; W[4 * j + 2] = v.z; W[4 * j + 3] = v.w; }
  }
  // slides the window until pos - cb < 16
  YDEV void advance(uint64_t pos) {
    while (pos - cb >= 16) {
#pragma unroll
      for (int j = 0; j < 12; j++) W[j] = W[j + 4];
      const u32x4 v = ld(cb + 64);
      W[12] = v.x; W[13] = v.y; W[14] = v.z; W[15] = v.w;
      cb += 16;
    }
  }
  // bytes pos .. pos+31 (pos - cb < 16) as 8 dwords
  YDEV void view(uint64_t pos, uint32_t (&d)[8]) const {
    const uint32_t r = (uint32_t)(pos - cb);
    const uint32_t m1 = 0u - ((r >> 2) & 1u), m2 = 0u - ((r >> 3) & 1u);
    uint32_t L[9];
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint32_t s0 = (W[j + 1] & m1) | (W[j] & ~m1);
      const uint32_t s1 = (W[j + 3] & m1) | (W[j + 2] & ~m1);
      L[j] = (s1 & m2) | (s0 & ~m2);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) d[j] = __builtin_amdgcn_alignbyte(L[j + 1], L[j], r & 3u);
  }
};

// masks of a 32-byte view: H = top bit, Z = zero byte ("haszero"), V = bytes inside the document
struct VMask { uint32_t H, Z, T, V; };
YDEV VMask vmask(const uint32_t (&d)[8], uint64_t rem) {
  VMask m; m.H = 0; m.Z = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    m.H |= top8(d[2 * j], d[2 * j + 1]) << (8 * j);
    const uint32_t z0 = (d[2 * j] - 0x01010101u) & ~d[2 * j], z1 = (d[2 * j + 1] - 0x01010101u) & ~d[2 * j + 1];
    m.Z |= top8(z0, z1) << (8 * j);
  }
  m.V = rem >= 32 ? 0xFFFFFFFFu : ((1u << (uint32_t)rem) - 1u);
  m.T = ~m.H & m.V & 0x7FFFFFFFu;   // (byte 31 is never taken as a terminator: vend() == 31 means "not in the view")
  return m;
}
// byte p (< 32) of a view
YDEV uint32_t vbyte(const uint32_t (&d)[8], uint32_t p) {
  const uint32_t q = p >> 2;
  const uint32_t a = (q & 1) ? d[1] : d[0], b = (q & 1) ? d[3] : d[2], c = (q & 1) ? d[5] : d[4], e = (q & 1) ? d[7] : d[6];
  const uint32_t x = (q & 2) ? b : a, y = (q & 2) ? e : c;
  return ((q & 4) ? y : x) >> (8u * (p & 3u)) & 0xFFu;
}
// 8 bytes at p (< 32; bytes past 31 read as 0)
YDEV uint64_t vword(const uint32_t (&d)[8], uint32_t p) {
  const uint64_t U0 = ((uint64_t)d[1] << 32) | d[0], U1 = ((uint64_t)d[3] << 32) | d[2];
  const uint64_t U2 = ((uint64_t)d[5] << 32) | d[4], U3 = ((uint64_t)d[7] << 32) | d[6];
  const uint32_t q = p >> 3, sh = (p & 7u) * 8u;
  const uint64_t lo = q == 0 ? U0 : q == 1 ? U1 : q == 2 ? U2 : U3;
  const uint64_t hi = q == 0 ? U1 : q == 1 ? U2 : q == 2 ? U3 : 0ull;
  return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
}
// terminator of the varuint at p: index e (>= 31 when none inside the view)
YDEV uint32_t vend(uint32_t T, uint32_t p) {
  const uint32_t pp = p < 31u ? p : 31u;
  return pp + (uint32_t)__builtin_ctz((T >> pp) | 0x80000000u);
}
// value of the varuint [p, e] (<= 5 bytes; bad when longer, >= 2^32 or not inside the view)
YDEV uint32_t vval(const uint32_t (&d)[8], uint32_t p, uint32_t e, uint32_t& bad) {
  const uint32_t n = e - p + 1u;
  bad |= e >= 31u ? 1u : 0u;
  const uint64_t w = vword(d, p < 31u ? p : 31u);
  bad |= (n > 5u ? 1u : 0u) | (n == 5u ? ((uint32_t)(w >> 32) & 0x70u) : 0u);
  return pext32((uint32_t)w, (uint32_t)(w >> 32) & 0xFFu, n);
}

// One struct decoded at pos (its first byte is d[0] & 0xFF).
struct LStruct {
  uint32_t kind;    // K_GC / K_SKIP / K_ITEM
  uint32_t info;
  uint32_t len;     // clock length (< 2^32)
  uint64_t end;     // absolute offset after the struct
  // Item fields for re-encoding with an offset (positions relative to pos)
  uint32_t ro_p, ro_e;     // right origin bytes [ro_p, ro_e) (0, 0 when absent)
  uint32_t c_p;            // content start
  uint32_t sbad;
};

// Decodes the struct at pos from a fresh view; long ASCII strings are verified by streaming
// through the window (which is advanced past them).  sbad != 0: the document is deferred.
// whole-view checks: a >= 7-byte run of top-bit bytes (a varuint of >= 8 bytes), or a zero byte
// right after a top-bit byte (a non-minimal varuint): the document defers
YDEV uint32_t vcheck(const VMask& m) {
  const uint32_t HV = m.H & m.V;
  const uint32_t h2 = HV & (HV >> 1), h4 = h2 & (h2 >> 2), h7 = h4 & (h4 >> 3);
  return h7 | (m.Z & (HV << 1) & m.V);
}

// The struct at pos, given the view d / masks m at pos (w advanced so that pos - cb < 16).
YDEV LStruct lean_struct_at(SWin& w, uint64_t pos, uint64_t doc_end, const uint32_t (&d)[8], const VMask& m) {
  LStruct s; s.kind = K_ITEM; s.len = 0; s.end = pos; s.ro_p = 0; s.ro_e = 0; s.c_p = 0; s.sbad = 0;
  const uint32_t HV = m.H & m.V;
  uint32_t bad = 0;
  const uint32_t info = d[0] & 0xFFu;
  s.info = info;
  bad |= (m.V & 1u) ^ 1u;
  uint32_t p = 1u, e;
  if (info == 10u || (info & 31u) == 0u) {          // Skip / GC: varuint length
    s.kind = info == 10u ? K_SKIP : K_GC;
    e = vend(m.T, p);
    s.len = vval(d, p, e, bad);
    bad |= s.len == 0u ? 1u : 0u;
    p = e + 1u;
  } else {
    const uint32_t ref = info & 31u;
    bad |= (ref != 1u && ref != 4u && ref != 7u) ? 1u : 0u;   // other content: the exact per-document kernel
    const uint32_t t0 = (m.T >> 1) | 0x80000000u, t1 = t0 & (t0 - 1u), t2 = t1 & (t1 - 1u), t3 = t2 & (t2 - 1u);
    const uint32_t e2 = 1u + (uint32_t)__builtin_ctz(t1 | 0x80000000u) + 1u;   // after the 2nd varuint
    const uint32_t e4 = 1u + (uint32_t)__builtin_ctz(t3 | 0x80000000u) + 1u;   // after the 4th
    if ((info & 0xC0u) == 0xC0u) { s.ro_p = e2; s.ro_e = e4; p = e4; bad |= e4 >= 32u ? 1u : 0u; }
    else if (info & 0x80u) { p = e2; bad |= e2 >= 32u ? 1u : 0u; }
    else if (info & 0x40u) { s.ro_p = 1u; s.ro_e = e2; p = e2; bad |= e2 >= 32u ? 1u : 0u; }
    else {   // parent: parentInfo 1 (y-key string) / 0 (id); then parentSub when bit 0x20
      const uint32_t pi = vbyte(d, p < 31u ? p : 31u); p++;
      if (pi == 1u) {
        const uint32_t L = vbyte(d, p < 31u ? p : 31u); p++;
        bad |= (L & ~31u) | ((32u - p - L) & 0x80000000u) | ((HV >> (p < 31u ? p : 31u)) & ((1u << (L & 31u)) - 1u));
        p += L & 31u;
      } else {
        bad |= pi;
        e = vend(m.T, p); bad |= e >= 31u ? 1u : 0u; p = e + 1u;
        e = vend(m.T, p); bad |= e >= 31u ? 1u : 0u; p = e + 1u;
      }
      if (info & 0x20u) {
        const uint32_t L = vbyte(d, p < 31u ? p : 31u); p++;
        bad |= (L & ~31u) | ((32u - p - L) & 0x80000000u) | ((HV >> (p < 31u ? p : 31u)) & ((1u << (L & 31u)) - 1u));
        p += L & 31u;
      }
    }
    if ((info & 0xC0u) && (info & 0x20u)) bad |= 1u;   // yjs drops the bit on re-encode: exact kernel
    s.c_p = p;
    e = vend(m.T, p);
    const uint32_t v = vval(d, p, e, bad);
    p = e + 1u;
    if (ref == 1u) { s.len = v; bad |= v == 0u ? 1u : 0u; }
    else if (ref == 7u) {
      s.len = 1u;
      bad |= v > 6u ? 1u : 0u;
      if (v == 3u || v == 5u) {   // XmlElement node name / XmlHook name
        const uint32_t L = vbyte(d, p < 31u ? p : 31u); p++;
        bad |= (L & ~31u) | ((32u - p - L) & 0x80000000u) | ((HV >> (p < 31u ? p : 31u)) & ((1u << (L & 31u)) - 1u));
        p += L & 31u;
      }
    } else {   // ContentString: v bytes of ASCII (UTF-16 length == byte length)
      s.len = v;
      bad |= v == 0u ? 1u : 0u;
      if (p + v <= 32u) { bad |= (HV >> (p < 31u ? p : 31u)) & (v >= 32u ? 0xFFFFFFFFu : ((1u << v) - 1u)); p += v; }
      else {
        // long string: stream its bytes [pos + p, pos + p + v) through the window, 16 at a time
        uint64_t q = pos + p;
        const uint64_t qe = q + v;
        bad |= qe > doc_end ? 1u : 0u;
        while (!bad && q < qe) {
          w.advance(q);
          uint32_t dd[8];
          w.view(q, dd);
          const uint64_t left = qe - q;
          const uint32_t nb = left >= 16 ? 16u : (uint32_t)left;
          uint32_t hb = 0;
#pragma unroll
          for (int j = 0; j < 4; j++) hb |= (dd[j] & 0x80808080u);
          if (nb < 16u) {   // mask the bytes past the string
            hb = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const uint32_t lo = 4u * j;
              const uint32_t keep = nb <= lo ? 0u : nb >= lo + 4u ? 0xFFFFFFFFu : ((1u << (8u * (nb - lo))) - 1u);
              hb |= dd[j] & 0x80808080u & keep;
            }
          }
          bad |= hb;
          q += nb;
        }
        p += v;
      }
    }
  }
  s.end = pos + p;
  bad |= s.end > doc_end ? 1u : 0u;
  s.sbad = bad;
  return s;
}

YDEV LStruct lean_doc_struct(SWin& w, uint64_t pos, uint64_t doc_end) {
  w.advance(pos);
  uint32_t d[8];
  w.view(pos, d);
  const VMask m = vmask(d, doc_end - pos);
  LStruct s = lean_struct_at(w, pos, doc_end, d, m);
  s.sbad |= vcheck(m);
  return s;
}

// ---- lane-private output writers (global memory)
YDEV uint64_t gw_vu(uint8_t* __restrict__ o, uint64_t t, uint64_t v) {
  while (v > 127u) { o[t++] = (uint8_t)(0x80u | (v & 127u)); v >>= 7; }
  o[t++] = (uint8_t)v;
  return t;
}
// copies n bytes from src to dst (both global, unaligned): batches of eight 16-byte pieces (eight
// loads in flight before the stores), then single pieces, the last one overlapping its predecessor
// (all inside [dst, dst + n)); short runs byte by byte
YDEV void gw_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t n) {
  if (n < 16) { for (uint64_t i = 0; i < n; i++) dst[i] = src[i]; return; }
  uint64_t o = 0;
  for (; o + 128 <= n; o += 128) {
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) __builtin_memcpy(&v[k], src + o + 16 * k, 16);
#pragma unroll
    for (int k = 0; k < 8; k++) __builtin_memcpy(dst + o + 16 * k, &v[k], 16);
  }
  for (; o + 16 <= n; o += 16) { u32x4 v; __builtin_memcpy(&v, src + o, 16); __builtin_memcpy(dst + o, &v, 16); }
  if (o < n) { u32x4 v; __builtin_memcpy(&v, src + n - 16, 16); __builtin_memcpy(dst + n - 16, &v, 16); }
}

// Re-encodes the struct at pos with `off` leading clock units removed (Item.write(encoder,
// off) / GC, Y@80416 / Y@68955) for the ASCII-only struct kinds lean_doc_struct accepts.
// Returns the new output position.
YDEV uint64_t lean_write_sliced(uint8_t* __restrict__ o, uint64_t t, const uint8_t* __restrict__ in, uint64_t pos, const LStruct& s,
                                uint32_t client, uint32_t clock, uint32_t off) {
  if (s.kind == K_GC) { o[t++] = 0; return gw_vu(o, t, s.len - off); }
  const uint32_t info = s.info, ref = info & 31u;
  const bool ho = (info & 0x80u) != 0, hr = (info & 0x40u) != 0;
  const bool has_sub = !ho && !hr && (info & 0x20u);   // yjs sets the bit, writes no parentSub (origin present)
  o[t++] = (uint8_t)(ref | 0x80u | (hr ? 0x40u : 0u) | (has_sub ? 0x20u : 0u));
  t = gw_vu(o, t, client);
  t = gw_vu(o, t, (uint64_t)clock + off - 1u);
  for (uint32_t i = s.ro_p; i < s.ro_e; i++) o[t++] = in[pos + i];   // right origin, verbatim (minimal varuints)
  if (ref == 1u) return gw_vu(o, t, s.len - off);
  // ContentString (ASCII): the content varuint starts at c_p
  uint32_t lb = 1; for (uint32_t v = s.len; v > 127u; v >>= 7) lb++;
  t = gw_vu(o, t, s.len - off);
  const uint64_t src = pos + s.c_p + lb + off;
  for (uint32_t i = 0; i < s.len - off; i++) o[t++] = in[src + i];
  return t;
}

}  // namespace ygm
