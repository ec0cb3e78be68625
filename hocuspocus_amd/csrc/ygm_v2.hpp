// ygm_v2.hpp -- device-side Yjs update-V2 codec for gfx950 kernels (ygm_v2.hip).
//
// An update V2 (yjs UpdateEncoderV2.toUint8Array, Y@18700 of the 13.5.16 bundle) is
//   varUint 0 | nine varUint8Array columns | rest
// with the columns keyClock (IntDiffOptRle), client (UintOptRle), leftClock, rightClock (IntDiffOptRle),
// info (Rle of bytes), string (varString of all strings joined + UintOptRle of their UTF-16 lengths),
// parentInfo (Rle of bytes), typeRef, len (UintOptRle), and the rest holding block headers, Skip lengths,
// Any / Buf content and the delete set (clocks diff-coded per client, lengths - 1).  lib0 0.2.42's coders:
// chunk 8086 of the bundle (decoders N / P / G / $, encoders $ / K / H / W).
//
// yjs's V2 functions are its V1 functions with V2 coders: the structs read and the writer calls made do
// not depend on the format.  The engine therefore transcodes, one lane per update:
//   v21  (UpdateDecoderV2 reads, V1 bytes out)   V2 -> V1, the same blocks / structs / info bytes /
//        delete-set entries.  ContentEmbed / ContentFormat values (an Any in V2, a JSON string in V1) are
//        carried as a placeholder number -- the Any's byte offset in the V2 arena, with a leading blank
//        when writeAny would not reproduce the Any so the V1 layer refuses the struct exactly when it
//        writes it -- or, for the public conversion, as JSON.stringify of the Any.
//   v12  (V1 bytes in, UpdateEncoderV2 writes)   yjs 13.6 convertUpdateFormat(V1 -> V2) on lazy-writer-
//        normal V1 (what the V1 merge / diff kernels emit; other V1 is refused by the public conversion).
// Both run a count pass (no stores) and a write pass at offsets from a scan.  The same rules as the CPU
// restatement oracle/yjs_oracle_v2.c, kept in lock-step by the parity tests; reads past a column's end keep
// JavaScript's `arr[pos++] === undefined` arithmetic.
#pragma once
#include "ygm_v1.hpp"
#ifdef YGM_HOST_BUILD
static inline uint32_t __float_as_uint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline long long __double_as_longlong(double x) { long long u; memcpy(&u, &x, 8); return u; }
#endif

namespace ygm {
namespace v2 {

constexpr int V2_UNDEF = -1;
constexpr uint32_t M_EXPORT = 1u;        // public conversion: real JSON, normal form required
constexpr uint32_t M_STRUCTS_ONLY = 2u;  // v21: structs only (encodeStateVectorFromUpdateV2), empty delete set

// ---------------------------------------------------------------- column decoders (lib0 0.2.42)
struct Col { const uint8_t* p; uint32_t n; uint64_t pos; };
YDEV uint32_t col_rdu(Col& c, int& err) {   // readVarUint `U`
  uint32_t s = 0; int n = 0;
  for (;;) {
    const bool have = c.pos < c.n; const uint32_t e = have ? c.p[c.pos] : 0u; c.pos++;
    if (have) s |= (e & 127u) << (n & 31);
    n += 7;
    if (have && e < 128) return s;
    if (n > 35) { if (!err) err = ST_MALFORMED; return 0; }
  }
}
YDEV uint32_t col_rdi(Col& c, bool& neg, int& err) {   // readVarInt `T`: magnitude + sign bit
  bool have = c.pos < c.n; uint32_t s = have ? c.p[c.pos] : 0u; c.pos++;
  uint32_t n = s & 63; neg = (s & 64) != 0;
  if (!(s & 128)) return n;
  int e = 6;
  for (;;) {
    have = c.pos < c.n; s = have ? c.p[c.pos] : 0u; c.pos++;
    if (have) n |= (s & 127u) << (e & 31);
    e += 7;
    if (have && s < 128) return n;
    if (e > 41) { if (!err) err = ST_MALFORMED; return 0; }
  }
}
struct RleD { Col c; int64_t count; int s; };
struct UoD { Col c; int64_t count; uint32_t s; };
struct IdD { Col c; int64_t count; int64_t s, diff; };
YDEV int rle_read(RleD& d, int& err) {
  if (d.count == 0) {
    const bool have = d.c.pos < d.c.n; d.s = have ? (int)d.c.p[d.c.pos] : V2_UNDEF; d.c.pos++;
    if (d.c.pos != d.c.n) d.count = (int64_t)col_rdu(d.c, err) + 1; else d.count = -1;   // hasContent
  }
  d.count--;
  return d.s;
}
YDEV uint32_t uo_read(UoD& d, int& err) {
  if (d.count == 0) {
    bool neg; d.s = col_rdi(d.c, neg, err); d.count = 1;
    if (neg) d.count = (int64_t)col_rdu(d.c, err) + 2;
  }
  d.count--;
  return d.s;
}
YDEV int64_t id_read(IdD& d, int& err) {
  if (d.count == 0) {
    bool neg; const uint32_t m = col_rdi(d.c, neg, err);
    const int32_t t = (int32_t)(neg ? 0u - m : m);
    d.diff = t >> 1; d.count = 1;
    if (t & 1) d.count = (int64_t)col_rdu(d.c, err) + 2;
  }
  d.s += d.diff;
  d.count--;
  return d.s;
}

struct Dec2 {
  Cur rest;
  IdD kc, lc, rc; UoD cl, tr, ln, lens; RleD info, pi;
  const uint8_t* str; uint32_t sn, sb;
  uint64_t nkeys;
  int err;
  YDEV void fail(int e) { if (!err) err = e; }
  YDEV int st() const { return err ? err : rest.err; }
};

YDEV void open2(Dec2& v, const uint8_t* u, uint32_t n, uint32_t flags) {
  v.rest = Cur{u, 0, n, 0, 0};
  v.err = 0; v.nkeys = 0; v.sb = 0; v.sn = 0; v.str = u;
  (void)v.rest.vu();
  Col cols[9];
  for (int i = 0; i < 9; i++) {
    uint32_t l; const uint32_t s = v.rest.buf(l);
    cols[i] = Col{u + s, l, 0};
    if (v.rest.err) return;
  }
  Col sc = cols[5]; int e = 0;
  const uint32_t sl = col_rdu(sc, e);
  if (e) { v.fail(e); return; }
  // lib0 0.2.42 readVarString: byte by byte when length - 1 < 100 (a missing byte throws), else in clamped
  // chunks that never throw; 0.2.104 reads a bounded view (always a throw)
  const uint32_t avail = sc.pos < sc.n ? sc.n - (uint32_t)sc.pos : 0u;
  if (sl > 0 && (avail == 0 || ((sl - 1 < 100 || !(flags & F_COMPAT_135)) && sl > avail))) { v.fail(ST_MALFORMED); return; }
  v.str = sc.p + sc.pos; v.sn = sl < avail ? sl : avail; sc.pos += sl;
  if (utf8_u16(v.str, v.sn) < 0) { v.fail(ST_MALFORMED); return; }
  v.kc = IdD{cols[0], 0, 0, 0}; v.cl = UoD{cols[1], 0, 0}; v.lc = IdD{cols[2], 0, 0, 0}; v.rc = IdD{cols[3], 0, 0, 0};
  v.info = RleD{cols[4], 0, 0}; v.lens = UoD{sc, 0, 0}; v.pi = RleD{cols[6], 0, 0}; v.tr = UoD{cols[7], 0, 0};
  v.ln = UoD{cols[8], 0, 0};
}
// StringDecoder.read: str.slice(spos, spos + len) at UTF-16 offsets; *len bytes at the returned pointer
YDEV const uint8_t* rd_string(Dec2& v, uint32_t& len) {
  int e = 0;
  uint64_t want = uo_read(v.lens, e);
  if (e) { v.fail(e); len = 0; return v.str; }
  const uint32_t b0 = v.sb;
  while (want > 0 && v.sb < v.sn) {
    const uint8_t ch = v.str[v.sb];
    const uint32_t k = ch < 0x80 ? 1u : (ch & 0xE0) == 0xC0 ? 2u : (ch & 0xF0) == 0xE0 ? 3u : 4u;
    if (k == 4) { if (want == 1) { v.fail(ST_NONCANON); len = 0; return v.str; } want -= 2; }   // splits a surrogate pair
    else want -= 1;
    v.sb += k;
  }
  len = v.sb - b0;
  return v.str + b0;
}
YDEV uint32_t rd_client(Dec2& v) { int e = 0; const uint32_t x = uo_read(v.cl, e); if (e) v.fail(e); return x; }
YDEV uint32_t rd_len(Dec2& v) { int e = 0; const uint32_t x = uo_read(v.ln, e); if (e) v.fail(e); return x; }
YDEV uint64_t rd_clock(Dec2& v, IdD& d) {
  int e = 0; const int64_t x = id_read(d, e);
  if (e) v.fail(e);
  if (x < 0 || (uint64_t)x > MAX_SAFE) { v.fail(ST_NONCANON); return 0; }   // a clock V1 cannot carry (hand-made input)
  return (uint64_t)x;
}

YDEV void vstr(Out& o, const uint8_t* s, uint32_t n) { o.vu(n); o.copy(s, n); }
YDEV uint32_t dec_digits(uint64_t v, uint8_t* t) {   // decimal, most significant first; returns the count
  uint8_t r[20]; uint32_t k = 0;
  do { r[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
  for (uint32_t i = 0; i < k; i++) t[i] = r[k - 1 - i];
  return k;
}

// ---------------------------------------------------------------- Any -> JSON.stringify (public V2 -> V1)
YDEV void js_quote(Out& o, const uint8_t* s, uint32_t n) {
  const char* hx = "0123456789abcdef";
  o.b('"');
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    if (c == '"' || c == '\\') { o.b('\\'); o.b(c); }
    else if (c == 8) { o.b('\\'); o.b('b'); } else if (c == 9) { o.b('\\'); o.b('t'); } else if (c == 10) { o.b('\\'); o.b('n'); }
    else if (c == 12) { o.b('\\'); o.b('f'); } else if (c == 13) { o.b('\\'); o.b('r'); }
    else if (c < 0x20) { o.b('\\'); o.b('u'); o.b('0'); o.b('0'); o.b((uint8_t)hx[c >> 4]); o.b((uint8_t)hx[c & 15]); }
    else o.b(c);
  }
  o.b('"');
}
// one canonical Any (validated) as JSON.stringify writes it; numbers other than varInt integers, undefined and
// Uint8Array are refused (ST_NONCANON), a BigInt throws in JSON.stringify (ST_MALFORMED)
YDEV_NI int any_json(Cur& c, Out& o) {
  uint32_t rem[MAX_DEPTH + 1]; uint8_t obj[MAX_DEPTH + 1]; uint8_t first[MAX_DEPTH + 1];
  int d = 0; rem[0] = 1; obj[0] = 2; first[0] = 1;
  while (!c.err) {
    if (rem[d] == 0) { if (d == 0) break; o.b(obj[d] == 1 ? '}' : ']'); d--; continue; }
    rem[d]--;
    if (obj[d] != 2) { if (!first[d]) o.b(','); first[d] = 0; }
    if (obj[d] == 1) {
      uint32_t kl; const uint32_t ks = c.buf(kl); if (c.err) break;
      js_quote(o, c.p + ks, kl); o.b(':');
      if (c.pos < c.end && c.p[c.pos] == 127) return ST_NONCANON;   // an undefined member: dropped by stringify
    }
    const uint8_t tag = c.u8();
    if (c.err) break;
    switch (tag) {
      case 126: o.b('n'); o.b('u'); o.b('l'); o.b('l'); break;
      case 120: o.b('t'); o.b('r'); o.b('u'); o.b('e'); break;
      case 121: o.b('f'); o.b('a'); o.b('l'); o.b('s'); o.b('e'); break;
      case 125: {
        const uint8_t r = c.u8(); uint64_t num = r & 63; uint32_t sh = 6;
        if (r & 128) for (;;) { const uint8_t b = c.u8(); if (c.err) break; if (sh < 60) num |= (uint64_t)(b & 127) << sh; sh += 7; if (b < 128) break; }
        if ((r & 64) && num) o.b('-');
        uint8_t t[20]; const uint32_t k = dec_digits(num, t); o.copy(t, k);
        break;
      }
      case 119: { uint32_t l; const uint32_t s = c.buf(l); if (!c.err) js_quote(o, c.p + s, l); break; }
      case 117: case 118: {
        const uint64_t n = c.vu(); if (c.err) break;
        if (d + 1 > MAX_DEPTH) return ST_DEPTH;
        o.b(tag == 118 ? '{' : '[');
        d++; rem[d] = (uint32_t)n; obj[d] = tag == 118; first[d] = 1;
        break;
      }
      case 122: return ST_MALFORMED;
      default: return ST_NONCANON;
    }
  }
  return c.err;
}

// ---------------------------------------------------------------- JSON.parse -> writeAny (public V1 -> V2)
// s is canonical (json_check without nc): no whitespace, keys without escapes, short escapes or \u00xx for
// control characters, numbers of <= 15 significant digits and no exponent -- so a number is M * 10^z or
// M / 10^f with M < 2^53 and z, f <= 22: one correctly rounded IEEE multiply / divide (Clinger's fast path).
YDEV void any_vi(Out& o, uint64_t m, bool neg) {   // lib0 writeVarInt of a magnitude < 2^32
  m &= 0xFFFFFFFFull;
  o.b((uint8_t)((m > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (m & 63)));
  m >>= 6;
  while (m > 0) { o.b((uint8_t)((m > 127 ? 0x80 : 0) | (m & 127))); m >>= 7; }
}
YDEV uint32_t json_str_body(const uint8_t* s, uint32_t n, uint32_t i, Out* o) {   // s[i] == '"'; decoded bytes
  uint32_t len = 0; i++;
  while (i < n && s[i] != '"') {
    uint8_t ch = s[i];
    if (ch == '\\') {
      const uint8_t e = s[i + 1];
      if (e == 'u') { ch = (uint8_t)(hexv(s[i + 2]) * 4096 + hexv(s[i + 3]) * 256 + hexv(s[i + 4]) * 16 + hexv(s[i + 5])); i += 6; }
      else { ch = e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e; i += 2; }
    } else i++;
    if (o) o->b(ch);
    len++;
  }
  return len;
}
YDEV uint32_t json_str_any(const uint8_t* s, uint32_t n, uint32_t i, Out& o) {   // writes varString; returns index after
  const uint32_t len = json_str_body(s, n, i, nullptr);
  o.vu(len);
  json_str_body(s, n, i, &o);
  i++;
  while (s[i] != '"') i += s[i] == '\\' ? (s[i + 1] == 'u' ? 6u : 2u) : 1u;
  return i + 1;
}
YDEV uint32_t json_num_any(const uint8_t* s, uint32_t n, uint32_t i, Out& o, uint32_t flags) {
  const double P10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15, 1e16,
                          1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  bool neg = false;
  if (s[i] == '-') { neg = true; i++; }
  // digits without the dot; an integer's trailing zeros become a power of ten (canonical: <= 15 significant)
  uint64_t m = 0; int frac = 0, tz = 0; bool dot = false;
  while (i < n) {
    const uint8_t ch = s[i];
    if (ch == '.') { for (; tz > 0; tz--) m *= 10; dot = true; i++; continue; }
    if (ch < '0' || ch > '9') break;
    const uint32_t dg = ch - '0';
    if (dot) { m = m * 10 + dg; frac++; }
    else if (dg == 0 && m != 0) tz++;
    else { for (; tz > 0; tz--) m *= 10; m = m * 10 + dg; }
    i++;
  }
  double x = (double)m;
  if (frac) x = x / P10[frac]; else if (tz) x = x * P10[tz];
  if (neg) x = -x;
  if (js_small_int(x, flags)) { o.b(125); const double ax = fabs(x); any_vi(o, (uint64_t)fmod(ax, 4294967296.0), x < 0); }
  else if ((double)(float)x == x) { const uint32_t u = __float_as_uint((float)x); o.b(124); for (int q = 3; q >= 0; q--) o.b((uint8_t)(u >> (8 * q))); }
  else { const uint64_t u = (uint64_t)__double_as_longlong(x); o.b(123); for (int q = 7; q >= 0; q--) o.b((uint8_t)(u >> (8 * q))); }
  return i;
}
// writeAny(JSON.parse(s)) for canonical s
YDEV_NI void json_to_any(const uint8_t* s, uint32_t n, Out& o, uint32_t flags) {
  uint32_t rem[MAX_DEPTH + 1]; uint8_t obj[MAX_DEPTH + 1];
  int d = 0; rem[0] = 1; obj[0] = 2;
  uint32_t i = 0;
  while (i < n || rem[d] == 0) {
    if (rem[d] == 0) { if (d == 0) break; i++; d--; if (rem[d] > 0) i++; continue; }   // the closing bracket (and a ',')
    rem[d]--;
    if (obj[d] == 1) { i = json_str_any(s, n, i, o); i++; }       // key, ':'
    const uint8_t c = s[i];
    if (c == '{' || c == '[') {
      uint32_t cnt = 0, j = i + 1; int dp = 0; bool in = false;
      if (s[j] != (c == '{' ? '}' : ']')) {
        cnt = 1;
        for (; j < n; j++) {
          const uint8_t ch = s[j];
          if (in) { if (ch == '\\') j++; else if (ch == '"') in = false; continue; }
          if (ch == '"') in = true;
          else if (ch == '{' || ch == '[') dp++;
          else if (ch == '}' || ch == ']') { if (dp == 0) break; dp--; }
          else if (ch == ',' && dp == 0) cnt++;
        }
      }
      o.b(c == '{' ? 118 : 117); o.vu(cnt);
      i++;
      if (d + 1 > MAX_DEPTH) return;
      d++; rem[d] = cnt; obj[d] = c == '{';
      continue;
    }
    if (c == '"') { o.b(119); i = json_str_any(s, n, i, o); }
    else if (c == 't') { o.b(120); i += 4; }
    else if (c == 'f') { o.b(121); i += 5; }
    else if (c == 'n') { o.b(126); i += 4; }
    else i = json_num_any(s, n, i, o, flags);
    if (rem[d] > 0) i++;   // ','
  }
}

// ---------------------------------------------------------------- V2 -> V1
// arena_off: the update's offset in the V2 arena (placeholders name absolute offsets)
// (pointer arguments on copies of the caller's state: a reference into Dec2 / Out would pin them in scratch)
YDEV_NI int v2_json(Cur* restp, Out* op, uint64_t arena_off, uint32_t mode, uint32_t flags) {
  Cur& rest = *restp; Out& o = *op;
  const uint32_t a = rest.pos; bool nc = false;
  any_value(rest, nc, flags);
  if (rest.err) return rest.err;
  if (!(mode & M_EXPORT)) {
    uint8_t t[21]; uint32_t k = 0;
    if (nc) t[k++] = ' ';
    k += dec_digits(arena_off + a, t + k);
    o.vu(k); o.copy(t, k);
    return ST_OK;
  }
  if (nc) return ST_NONCANON;
  Cur q{rest.p, a, rest.pos, 0, 0};
  Out m{nullptr, 0};
  int e = any_json(q, m);
  if (e) return e;
  o.vu(m.n);
  Cur q2{rest.p, a, rest.pos, 0, 0};
  return any_json(q2, o);
}
YDEV int v2_json_call(Dec2& v, Out& o, uint64_t arena_off, uint32_t mode, uint32_t flags) {
  Cur r = v.rest; Out oo = o;
  const int e = v2_json(&r, &oo, arena_off, mode, flags);
  v.rest = r; o = oo;
  return e;
}
YDEV void any_value_call(Cur& c, bool& nc, uint32_t flags) { Cur q = c; bool n2 = nc; any_value(q, n2, flags); c = q; nc = n2; }

YDEV int v21(const uint8_t* u, uint32_t n, uint64_t arena_off, uint32_t mode, uint32_t flags, Out& o) {
  Dec2 v;
  open2(v, u, n, flags);
  if (v.st()) return v.st();
  // the public conversion (M_EXPORT) emits what convertUpdateFormat's lazy writer would: V2 input that is not
  // already in that normal form (empty or repeated-client blocks, info bits the writer recomputes, a delete
  // set readDeleteSet / writeDeleteSet would rewrite) is refused
  const bool ex = (mode & M_EXPORT) != 0;
  bool nonnormal = false;
  const uint64_t nb = v.rest.vu(); o.vu(nb);
  uint64_t prev = ~0ull;
  for (uint64_t b = 0; b < nb && !v.st(); b++) {
    const uint64_t ns = v.rest.vu(); const uint32_t client = rd_client(v); const uint64_t clock = v.rest.vu();
    if (v.st()) break;
    if (ns == 0 || client == prev) nonnormal = true;
    prev = client;
    o.vu(ns); o.vu(client); o.vu(clock);
    for (uint64_t s = 0; s < ns && !v.st(); s++) {
      int e = 0; const int info = rle_read(v.info, e);
      if (e) { v.fail(e); break; }
      if (info == 10) { const uint64_t l = v.rest.vu(); o.b(10); o.vu(l); continue; }
      if (info == V2_UNDEF || (info & 31) == 0) { if (info) nonnormal = true; o.b(0); o.vu(rd_len(v)); continue; }   // GC
      if ((info & 0xC0) && (info & 0x20)) nonnormal = true;   // parentSub bit beside an origin: not re-written
      o.b((uint8_t)info);
      if (info & 0x80) { o.vu(rd_client(v)); o.vu(rd_clock(v, v.lc)); }
      if (info & 0x40) { o.vu(rd_client(v)); o.vu(rd_clock(v, v.rc)); }
      if ((info & 0xC0) == 0) {
        const int p = rle_read(v.pi, e); if (e) { v.fail(e); break; }
        if (p == 1) { uint32_t l; const uint8_t* t = rd_string(v, l); o.b(1); vstr(o, t, l); }
        else { o.b(0); o.vu(rd_client(v)); o.vu(rd_clock(v, v.lc)); }
        if (info & 0x20) { uint32_t l; const uint8_t* t = rd_string(v, l); vstr(o, t, l); }
      }
      if (v.st()) break;
      switch (info & 31) {
        case 1: o.vu(rd_len(v)); break;                                                     // ContentDeleted
        case 2: {                                                                           // ContentJSON
          const uint32_t k = rd_len(v); o.vu(k);
          for (uint32_t i = 0; i < k && !v.st(); i++) {
            uint32_t l; const uint8_t* t = rd_string(v, l); if (v.st()) break; vstr(o, t, l);
            if (!(l == 9 && t[0] == 'u' && t[1] == 'n' && t[2] == 'd' && t[3] == 'e' && t[4] == 'f' && t[5] == 'i' && t[6] == 'n' &&
                  t[7] == 'e' && t[8] == 'd')) {
              bool nc = false; const int je = json_check(t, l, nc); if (je) v.fail(je);
            }
          }
          break;
        }
        case 3: { uint32_t l; const uint32_t st = v.rest.buf(l); if (!v.rest.err) vstr(o, u + st, l); break; }   // ContentBinary
        case 4: { uint32_t l; const uint8_t* t = rd_string(v, l); vstr(o, t, l); break; }                      // ContentString
        case 5: { const int je = v2_json_call(v, o, arena_off, mode, flags); if (je) v.fail(je); break; }          // ContentEmbed
        case 6: {                                                                                              // ContentFormat
          uint32_t l; const uint8_t* t = rd_string(v, l); if (v.st()) break; vstr(o, t, l);
          const int je = v2_json_call(v, o, arena_off, mode, flags); if (je) v.fail(je);
          break;
        }
        case 7: {                                                                                              // ContentType
          const uint32_t tr = uo_read(v.tr, e); if (e) { v.fail(e); break; }
          if (tr > 6) { v.fail(ST_MALFORMED); break; }
          o.vu(tr);
          if (tr == 3 || tr == 5) {   // readKey: a cache hit (hand-made input) is refused
            const int64_t kc = id_read(v.kc, e); if (e) { v.fail(e); break; }
            if (kc < 0 || (uint64_t)kc < v.nkeys) { v.fail(ST_NONCANON); break; }
            uint32_t l; const uint8_t* t = rd_string(v, l); vstr(o, t, l); v.nkeys++;
          }
          break;
        }
        case 8: {                                                                                              // ContentAny
          const uint32_t k = rd_len(v); o.vu(k);
          const uint32_t a = v.rest.pos; bool nc = false;
          for (uint32_t i = 0; i < k && !v.st(); i++) any_value_call(v.rest, nc, flags);
          if (!v.st()) o.copy(u + a, v.rest.pos - a);
          break;
        }
        case 9: {                                                                                              // ContentDoc
          uint32_t l; const uint8_t* t = rd_string(v, l); if (v.st()) break; vstr(o, t, l);
          const uint32_t a = v.rest.pos; bool nc = false; any_value_call(v.rest, nc, flags);
          if (!v.st()) o.copy(u + a, v.rest.pos - a);
          break;
        }
        default: v.fail(ST_MALFORMED); break;
      }
    }
  }
  if (v.st()) return v.st();
  if (mode & M_STRUCTS_ONLY) { o.b(0); return ST_OK; }
  const uint64_t nc = v.rest.vu(); o.vu(nc);
  const uint32_t ds0 = v.rest.pos;
  uint64_t last = ~0ull;
  for (uint64_t i = 0; i < nc && !v.st(); i++) {
    uint64_t cur = 0;
    const uint64_t client = v.rest.vu(), nd = v.rest.vu();
    if (v.st()) break;
    if (ex) {
      if (nd == 0 || (!(flags & F_COMPAT_135) && i > 0 && client >= last)) nonnormal = true;
      else if (flags & F_COMPAT_135) {   // distinct clients (readDeleteSet joins repeats)
        Cur r{u, ds0, n, 0, 0};
        for (uint64_t j = 0; j < i; j++) { const uint64_t cj = r.vu(), nj = r.vu(); if (cj == client) nonnormal = true; for (uint64_t k = 0; k < 2 * nj; k++) r.vu(); }
      }
    }
    last = client;
    o.vu(client); o.vu(nd);
    for (uint64_t k = 0; k < nd && !v.st(); k++) {
      cur += v.rest.vu(); const uint64_t clock = cur;
      const uint64_t len = v.rest.vu() + 1; cur += len;
      if (cur > MAX_SAFE) { v.fail(ST_RANGE); break; }
      o.vu(clock); o.vu(len);
    }
  }
  if (v.st()) return v.st();
  return ex && nonnormal ? ST_NONCANON : ST_OK;
}

// ---------------------------------------------------------------- V1 -> V2
struct RleE { int64_t count; int s; };
struct UoE { int64_t count; uint64_t s; };
struct IdE { int64_t count; int64_t s, diff; };
YDEV void rle_w(Out& o, RleE& e, int v) {
  if (e.s == v) { e.count++; return; }
  if (e.count > 0) o.vu((uint64_t)(e.count - 1));
  e.count = 1; o.b((uint8_t)v); e.s = v;
}
YDEV void uo_flush(Out& o, const UoE& e) {
  if (e.count > 0) { any_vi(o, e.s, e.count != 1); if (e.count > 1) o.vu((uint64_t)(e.count - 2)); }
}
YDEV void uo_w(Out& o, UoE& e, uint64_t v) { if (e.s == v) { e.count++; return; } uo_flush(o, e); e.count = 1; e.s = v; }
YDEV void id_flush(Out& o, const IdE& e) {
  if (e.count > 0) {
    const int32_t v = (int32_t)(((uint32_t)(uint64_t)e.diff << 1) | (e.count == 1 ? 0u : 1u));   // diff << 1 | run, int32
    any_vi(o, v < 0 ? (uint64_t)(0u - (uint32_t)v) : (uint64_t)v, v < 0);
    if (e.count > 1) o.vu((uint64_t)(e.count - 2));
  }
}
YDEV void id_w(Out& o, IdE& e, int64_t v) { if (e.diff == v - e.s) { e.s = v; e.count++; return; } id_flush(o, e); e.count = 1; e.diff = v - e.s; e.s = v; }

enum { C_KC, C_CL, C_LC, C_RC, C_INFO, C_STR, C_LENS, C_PI, C_TR, C_LN, C_REST, C_N };
struct Enc2 {
  Out o[C_N];
  IdE kc, lc, rc; UoE cl, tr, ln, lens; RleE info, pi;
  uint64_t keyclock;
};
YDEV void e_str(Enc2& w, const uint8_t* s, uint32_t n) { w.o[C_STR].copy(s, n); uo_w(w.o[C_LENS], w.lens, (uint64_t)utf8_u16(s, n)); }
YDEV void e_key(Enc2& w, const uint8_t* s, uint32_t n) { id_w(w.o[C_KC], w.kc, (int64_t)w.keyclock++); e_str(w, s, n); }
// writeJSON: the placeholder's Any bytes from the V2 arena, or writeAny(JSON.parse(s))
YDEV_NI int e_json(Out* restp, const uint8_t* s, uint32_t n, const uint8_t* v2a, uint64_t v2n, uint32_t mode, uint32_t flags) {
  Out& rest = *restp;
  if (!(mode & M_EXPORT)) {
    uint32_t i = 0; while (i < n && s[i] == ' ') i++;
    uint64_t at = 0; for (; i < n; i++) at = at * 10 + (s[i] - '0');
    if (at >= v2n) return ST_MALFORMED;
    Cur q{v2a + at, 0, (uint32_t)((v2n - at) < 0xFFFFFFFFull ? (v2n - at) : 0xFFFFFFFFull), 0, 0};
    any_skip(q);
    rest.copy(v2a + at, q.pos);
    return ST_OK;
  }
  json_to_any(s, n, rest, flags);
  return ST_OK;
}
YDEV int e_json_call(Enc2& w, const uint8_t* s, uint32_t n, const uint8_t* v2a, uint64_t v2n, uint32_t mode, uint32_t flags) {
  Out r = w.o[C_REST];
  const int e = e_json(&r, s, n, v2a, v2n, mode, flags);
  w.o[C_REST] = r;
  return e;
}

// v12 over one V1 update (lazy-writer normal: every block non-empty, consecutive blocks of different clients;
// export mode also requires a normal delete set: distinct clients with ranges, descending in 13.6 mode).
// Count pass: w.o[*].p == nullptr, the column lengths are w.o[*].n after the final flushes.
YDEV int v12_body(const uint8_t* p, uint32_t n, const uint8_t* v2a, uint64_t v2n, uint32_t mode, uint32_t flags, Enc2& w) {
  Cur c{p, 0, n, 0, 0};
  Out& rest = w.o[C_REST];
  const uint64_t nb = c.vu(); rest.vu(nb);
  uint64_t prev = ~0ull;
  bool nonnormal = false;
  for (uint64_t b = 0; b < nb && !c.err; b++) {
    const uint64_t ns = c.vu(), client = c.vu(), clock = c.vu();
    if (c.err) break;
    if (ns == 0 || client == prev) nonnormal = true;
    prev = client;
    uo_w(w.o[C_CL], w.cl, client); rest.vu(ns); rest.vu(clock);
    for (uint64_t s = 0; s < ns && !c.err; s++) {
      SInfo si; { Cur cc = c; read_struct(cc, si, flags); c = cc; }
      if (c.err) break;
      if (si.kind == K_GC) { rle_w(w.o[C_INFO], w.info, 0); uo_w(w.o[C_LN], w.ln, si.len); continue; }
      if (si.kind == K_SKIP) { rle_w(w.o[C_INFO], w.info, 10); rest.vu(si.len); continue; }
      if (si.nc) return ST_NONCANON;
      Cur h{p, si.start + 1, si.cstart, 0, 0};
      const uint8_t info = si.info;
      const bool ho = (info & 0x80) != 0, hr = (info & 0x40) != 0, hs = !ho && !hr && (info & 0x20);
      rle_w(w.o[C_INFO], w.info, (si.ref & 31) | (ho ? 0x80 : 0) | (hr ? 0x40 : 0) | (hs ? 0x20 : 0));
      if (ho) { const uint64_t oc = h.vu(), ok = h.vu(); uo_w(w.o[C_CL], w.cl, oc); id_w(w.o[C_LC], w.lc, (int64_t)ok); }
      if (hr) { const uint64_t rc = h.vu(), rk = h.vu(); uo_w(w.o[C_CL], w.cl, rc); id_w(w.o[C_RC], w.rc, (int64_t)rk); }
      if (!ho && !hr) {
        const uint64_t pi = h.vu();
        if (pi == 1) { rle_w(w.o[C_PI], w.pi, 1); uint32_t l; const uint32_t st = h.buf(l); e_str(w, p + st, l); }
        else { rle_w(w.o[C_PI], w.pi, 0); const uint64_t pc = h.vu(), pk = h.vu(); uo_w(w.o[C_CL], w.cl, pc); id_w(w.o[C_LC], w.lc, (int64_t)pk); }
        if (hs) { uint32_t l; const uint32_t st = h.buf(l); e_str(w, p + st, l); }
      }
      Cur q{p, si.cstart, si.end, 0, 0};
      switch (si.ref) {
        case 1: uo_w(w.o[C_LN], w.ln, q.vu()); break;
        case 2: { const uint64_t k = q.vu(); uo_w(w.o[C_LN], w.ln, k); for (uint64_t i = 0; i < k; i++) { uint32_t l; const uint32_t st = q.buf(l); e_str(w, p + st, l); } break; }
        case 3: { uint32_t l; const uint32_t st = q.buf(l); vstr(rest, p + st, l); break; }
        case 4: { uint32_t l; const uint32_t st = q.buf(l); e_str(w, p + st, l); break; }
        case 5: { uint32_t l; const uint32_t st = q.buf(l); const int e = e_json_call(w, p + st, l, v2a, v2n, mode, flags); if (e) return e; break; }
        case 6: {
          uint32_t l; uint32_t st = q.buf(l); e_key(w, p + st, l);
          st = q.buf(l); const int e = e_json_call(w, p + st, l, v2a, v2n, mode, flags); if (e) return e;
          break;
        }
        case 7: { const uint64_t tr = q.vu(); uo_w(w.o[C_TR], w.tr, tr); if (tr == 3 || tr == 5) { uint32_t l; const uint32_t st = q.buf(l); e_key(w, p + st, l); } break; }
        case 8: { const uint64_t k = q.vu(); uo_w(w.o[C_LN], w.ln, k); rest.copy(p + q.pos, si.end - q.pos); break; }
        case 9: { uint32_t l; const uint32_t st = q.buf(l); e_str(w, p + st, l); rest.copy(p + q.pos, si.end - q.pos); break; }
        default: return ST_MALFORMED;
      }
    }
  }
  if (c.err) return c.err;
  // readDeleteSet (V1) -> writeDeleteSet (V2)
  const uint64_t nd = c.vu(); if (c.err) return c.err;
  rest.vu(nd);
  uint64_t last = ~0ull;
  const uint32_t ds0 = c.pos;
  for (uint64_t i = 0; i < nd && !c.err; i++) {
    const uint64_t client = c.vu(), nr = c.vu();
    if (c.err) break;
    if (mode & M_EXPORT) {
      if (nr == 0 || (!(flags & F_COMPAT_135) && i > 0 && client >= last)) nonnormal = true;
      else if (flags & F_COMPAT_135) {   // distinct clients (readDeleteSet joins repeats)
        Cur r{p, ds0, n, 0, 0};
        for (uint64_t j = 0; j < i; j++) { const uint64_t cj = r.vu(), nj = r.vu(); if (cj == client) nonnormal = true; for (uint64_t k = 0; k < 2 * nj; k++) r.vu(); }
      }
    }
    last = client;
    rest.vu(client); rest.vu(nr);
    uint64_t cur = 0;
    for (uint64_t k = 0; k < nr && !c.err; k++) {
      const uint64_t clock = c.vu(), len = c.vu();
      if (c.err) break;
      if (clock >= cur) rest.vu(clock - cur); else rest.b((uint8_t)((clock - cur) & 127));   // writeVarUint(negative): one byte
      if (len == 0) return ST_MALFORMED;   // writeDsLen(0): unexpectedCase
      rest.vu(len - 1);
      cur = clock + len;
    }
  }
  if (c.err) return c.err;
  if (nonnormal) return ST_NONCANON;
  id_flush(w.o[C_KC], w.kc); uo_flush(w.o[C_CL], w.cl); id_flush(w.o[C_LC], w.lc); id_flush(w.o[C_RC], w.rc);
  uo_flush(w.o[C_LENS], w.lens); uo_flush(w.o[C_TR], w.tr); uo_flush(w.o[C_LN], w.ln);
  return ST_OK;
}
YDEV void enc_init(Enc2& w) {
  for (int i = 0; i < C_N; i++) w.o[i] = Out{nullptr, 0};
  w.kc = IdE{0, 0, 0}; w.lc = IdE{0, 0, 0}; w.rc = IdE{0, 0, 0};
  w.cl = UoE{0, 0}; w.tr = UoE{0, 0}; w.ln = UoE{0, 0}; w.lens = UoE{0, 0};
  w.info = RleE{0, -1}; w.pi = RleE{0, -1};
  w.keyclock = 0;
}
// total V2 size from the column lengths (UpdateEncoderV2.toUint8Array layout)
YDEV uint64_t v2_total(const uint32_t* L) {
  uint64_t t = 1;
  const int cols[8] = {C_KC, C_CL, C_LC, C_RC, C_INFO, C_PI, C_TR, C_LN};
  for (int q = 0; q < 8; q++) t += vu_len(L[cols[q]]) + L[cols[q]];
  const uint64_t sc = vu_len(L[C_STR]) + (uint64_t)L[C_STR] + L[C_LENS];
  return t + vu_len(sc) + sc + L[C_REST];
}
// write pass: headers at dst, each column's Out placed at its final offset, then the same encoding
YDEV int v12_write(const uint8_t* p, uint32_t n, const uint8_t* v2a, uint64_t v2n, uint32_t mode, uint32_t flags,
                      const uint32_t* L, uint8_t* dst) {
  Enc2 w; enc_init(w);
  Out h{dst, 0};
  h.b(0);
  uint8_t* cp[C_N];
  const int pre[5] = {C_KC, C_CL, C_LC, C_RC, C_INFO}, post[3] = {C_PI, C_TR, C_LN};
  for (int q = 0; q < 5; q++) { const int i = pre[q]; h.vu(L[i]); cp[i] = dst + h.n; h.n += L[i]; }
  const uint64_t sc = vu_len(L[C_STR]) + (uint64_t)L[C_STR] + L[C_LENS];
  h.vu(sc); h.vu(L[C_STR]);
  cp[C_STR] = dst + h.n; h.n += L[C_STR];
  cp[C_LENS] = dst + h.n; h.n += L[C_LENS];
  for (int q = 0; q < 3; q++) { const int i = post[q]; h.vu(L[i]); cp[i] = dst + h.n; h.n += L[i]; }
  cp[C_REST] = dst + h.n;
  for (int i = 0; i < C_N; i++) w.o[i] = Out{cp[i], 0};
  return v12_body(p, n, v2a, v2n, mode, flags, w);
}

}  // namespace v2
}  // namespace ygm
