// ygm_v1.hpp -- device-side Yjs update-v1 codec for gfx950 kernels.
//
// Byte format: SURVEY.md App. A (read from yjs Y@14063-17300 V1 coders,
// Y@36564 lazy struct reader, Y@80416 Item.write, Y@81141 content table and
// lib0 L0@2955-4074 / L0@7250-8700).  Everything here is a __device__ inline
// helper used by the kernels in ygm_kernels.hip; nothing allocates.
//
// Conventions
//  * A `Cur` walks one document-relative byte window [0, end) of global memory.
//    Any read past `end` fails with ST_MALFORMED (yjs/lib0 throw there too).
//  * Every loop whose trip count comes from the input also tests `c.err`, so a
//    corrupt count can never spin a wave.
//  * Content is validated the way yjs decodes it (TextDecoder{fatal}, readAny,
//    JSON.parse) and flagged NONCANON when yjs's re-encode (writeAny,
//    JSON.stringify) would produce different bytes (SURVEY.md App. A
//    "Canonical writers", App. C-9).  The rules are the same ones the CPU
//    oracle applies (oracle/yjs_oracle.c), kept in lock-step by the parity
//    tests.
#pragma once
#include <stdint.h>
#ifdef YGM_HOST_BUILD   // host build of the codec for development harnesses (tools/snapdev.cpp); kernels never use it
#include <string.h>
#include <math.h>
#define YDEV inline
#define YDEV_NI inline
static inline float __uint_as_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline double __longlong_as_double(long long u) { double f; memcpy(&f, &u, 8); return f; }
#else
#include <hip/hip_runtime.h>
#define YDEV __device__ __forceinline__
#define YDEV_NI __device__ __noinline__  // large, rarely-hot helpers: keep compile time and I-cache sane
#endif

namespace ygm {

enum : int {
  ST_OK = 0, ST_MALFORMED = 1, ST_RANGE = 2, ST_NONCANON = 3, ST_SURROGATE = 4, ST_DEPTH = 5,
  ST_NOMEM = 6, ST_DEVICE = 7, ST_INVAL = 8,
  ST_FALLBACK = 100  // internal: document must take the exact sequential kernel
};
enum : int { K_GC = 0, K_SKIP = 1, K_ITEM = 2 };
constexpr uint64_t MAX_SAFE = 9007199254740991ull;  // Number.MAX_SAFE_INTEGER (lib0 0.2.104 readVarUint)
constexpr int MAX_DEPTH = 32;                       // YGM_MAX_DEPTH
constexpr int MAX_KEYS = 64;                        // keys tracked per Any/JSON nesting stack
constexpr uint32_t F_COMPAT_135 = 1u;
// diff: every struct keeps its input's parentSub bit 0x20 (Item.write of an integrated item, Y@80416): the bytes
// Y.encodeStateAsUpdate(doc, sv) writes for a document loaded from a normalized state (ygm_sync_step2_v1)
constexpr uint32_t F_KEEP_SUB = 4u;

struct Cur {
  const uint8_t* p;
  uint32_t pos, end;
  int err;
  int nm;  // saw a non-minimal varuint
  YDEV void fail(int e) { if (!err) err = e; pos = end; }
  YDEV uint8_t u8() {
    if (pos >= end) { fail(ST_MALFORMED); return 0; }
    return p[pos++];
  }
  // lib0 readVarUint, 0.2.104 semantics (throws past 2^53)
  YDEV uint64_t vu() {
    uint64_t num = 0; uint32_t shift = 0;
    for (;;) {
      if (pos >= end) { fail(ST_MALFORMED); return 0; }
      const uint8_t r = p[pos++];
      if (shift < 63) num |= (uint64_t)(r & 127) << shift;
      else if (r & 127) { fail(ST_RANGE); return 0; }
      shift += 7;
      if (r < 128) {
        if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
        if (r == 0 && shift > 7) nm = 1;
        return num;
      }
      if (num > MAX_SAFE) { fail(ST_RANGE); return 0; }
    }
  }
  // readVarUint8Array: returns start, sets len; bounds checked
  YDEV uint32_t buf(uint32_t& len) {
    const uint64_t n = vu();
    if (err) { len = 0; return pos; }
    if (n > (uint64_t)(end - pos)) { fail(ST_MALFORMED); len = 0; return pos; }
    const uint32_t s = pos; pos += (uint32_t)n; len = (uint32_t)n; return s;
  }
};

YDEV uint32_t vu_len(uint64_t v) { uint32_t n = 1; while (v > 127) { v >>= 7; n++; } return n; }

// Strict UTF-8 (TextDecoder{fatal:true}); returns UTF-16 length or -1.
YDEV_NI int64_t utf8_u16(const uint8_t* s, uint32_t n) {
  int64_t u16 = 0; uint32_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80) { i++; u16++; continue; }
    int k; uint32_t cp, mn;
    if ((c & 0xE0) == 0xC0) { k = 1; cp = c & 0x1F; mn = 0x80; }
    else if ((c & 0xF0) == 0xE0) { k = 2; cp = c & 0x0F; mn = 0x800; }
    else if ((c & 0xF8) == 0xF0) { k = 3; cp = c & 0x07; mn = 0x10000; }
    else return -1;
    if (i + (uint32_t)k >= n) return -1;
    for (int j = 1; j <= k; j++) {
      const uint8_t cc = s[i + j];
      if ((cc & 0xC0) != 0x80) return -1;
      cp = (cp << 6) | (cc & 0x3F);
    }
    if (cp < mn || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return -1;
    u16 += cp >= 0x10000 ? 2 : 1;
    i += (uint32_t)k + 1;
  }
  return u16;
}

YDEV uint32_t str_hash(const uint8_t* s, uint32_t n) {  // FNV-1a 32
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < n; i++) { h ^= s[i]; h *= 16777619u; }
  return h ^ n;
}
// canonical array-index key (uint32 < 2^32-1): JS orders these first, ascending
YDEV bool index_key(const uint8_t* k, uint32_t n, uint64_t& v) {
  if (n == 0 || n > 10 || (n > 1 && k[0] == '0')) return false;
  v = 0;
  for (uint32_t i = 0; i < n; i++) { if (k[i] < '0' || k[i] > '9') return false; v = v * 10 + (k[i] - '0'); }
  return v < 4294967295ull;
}

// Own-property-order checks for one object level (Object.keys after obj[key]=v
// assignments / JSON.parse): index keys ascending and first, no duplicates.
// Duplicate detection compares 32-bit key hashes; a collision is refused as
// NONCANON (conservative).  The nesting state is kept as small per-level arrays
// (struct of arrays), sized by the caller: the full stack (MAX_DEPTH levels,
// MAX_KEYS keys: the sequential kernel and host code) or the register stack of the
// parallel tiers (SM_DEPTH levels, SM_KEYS keys: a value that needs more sends the
// document to the sequential kernel, ST_FALLBACK).
constexpr int SM_DEPTH = 4, SM_KEYS = 8;
// full stack: arrays (the sequential kernel's private memory, host code)
template <int D, int K>
struct AnyStack {
  uint32_t rem[D + 1], obj[D + 1], base[D + 1], seen[D + 1], hidx[D + 1];
  uint64_t lidx[D + 1];
  uint32_t h[K];
  int top = 0;
  YDEV uint32_t rget(int d) const { return rem[d]; }
  YDEV void rset(int d, uint32_t v) { rem[d] = v; }
  YDEV uint32_t oget(int d) const { return obj[d]; }
  YDEV void oset(int d, uint32_t v) { obj[d] = v; }
  YDEV void close_obj(int d) { top = (int)base[d]; }
  YDEV void open_obj(int d) { base[d] = (uint32_t)top; seen[d] = 0; hidx[d] = 0; lidx[d] = 0; }
  // returns 0 canonical so far, 1 noncanon
  YDEV int key(int d, const uint8_t* k, uint32_t n) {
    int r = 0;
    uint64_t v;
    if (index_key(k, n, v)) {
      if (seen[d] || (hidx[d] && v <= lidx[d])) r = 1;
      hidx[d] = 1; lidx[d] = v;
    } else seen[d] = 1;
    const uint32_t hh = str_hash(k, n);
    for (int i = (int)base[d]; i < top; i++) if (h[i] == hh) r = 1;
    if (top >= K) return 1;
    h[top++] = hh;
    return r;
  }
};
// register stack of the parallel tiers (SM_DEPTH levels, SM_KEYS keys): scalars selected by level, no private
// memory; key() returns 2 past SM_KEYS keys (the caller fails with ST_FALLBACK)
template <>
struct AnyStack<SM_DEPTH, SM_KEYS> {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
  uint64_t meta = 0;                      // per level 8 bits: 1 object, 2 string key seen, 4 index key seen, base << 4
  uint64_t l0 = 0, l1 = 0, l2 = 0, l3 = 0, l4 = 0;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0, h5 = 0, h6 = 0, h7 = 0;
  int top = 0;
  YDEV uint32_t rget(int d) const { return d == 0 ? r0 : d == 1 ? r1 : d == 2 ? r2 : d == 3 ? r3 : r4; }
  YDEV void rset(int d, uint32_t v) { r0 = d == 0 ? v : r0; r1 = d == 1 ? v : r1; r2 = d == 2 ? v : r2; r3 = d == 3 ? v : r3; r4 = d == 4 ? v : r4; }
  YDEV uint32_t mget(int d) const { return (uint32_t)(meta >> (8 * d)) & 0xFFu; }
  YDEV void mset(int d, uint32_t v) { meta = (meta & ~(0xFFull << (8 * d))) | ((uint64_t)(v & 0xFFu) << (8 * d)); }
  YDEV uint32_t oget(int d) const { return mget(d) & 1u; }
  YDEV void oset(int d, uint32_t v) { mset(d, (mget(d) & ~1u) | (v ? 1u : 0u)); }
  YDEV uint64_t lget(int d) const { return d == 0 ? l0 : d == 1 ? l1 : d == 2 ? l2 : d == 3 ? l3 : l4; }
  YDEV void lset(int d, uint64_t v) { l0 = d == 0 ? v : l0; l1 = d == 1 ? v : l1; l2 = d == 2 ? v : l2; l3 = d == 3 ? v : l3; l4 = d == 4 ? v : l4; }
  YDEV void close_obj(int d) { top = (int)(mget(d) >> 4); }
  YDEV void open_obj(int d) { mset(d, (mget(d) & 1u) | ((uint32_t)top << 4)); lset(d, 0); }
  YDEV int key(int d, const uint8_t* k, uint32_t n) {
    int r = 0;
    uint64_t v;
    uint32_t m = mget(d);
    if (index_key(k, n, v)) {
      if ((m & 2u) || ((m & 4u) && v <= lget(d))) r = 1;
      m |= 4u; lset(d, v);
    } else m |= 2u;
    mset(d, m);
    const uint32_t hh = str_hash(k, n);
    const int b = (int)(m >> 4);
    const uint32_t hs[8] = {h0, h1, h2, h3, h4, h5, h6, h7};
#pragma unroll
    for (int i = 0; i < 8; i++) if (i >= b && i < top && hs[i] == hh) r = 1;
    if (top >= SM_KEYS) return 2;
    h0 = top == 0 ? hh : h0; h1 = top == 1 ? hh : h1; h2 = top == 2 ? hh : h2; h3 = top == 3 ? hh : h3;
    h4 = top == 4 ? hh : h4; h5 = top == 5 ? hh : h5; h6 = top == 6 ? hh : h6; h7 = top == 7 ? hh : h7;
    top++;
    return r;
  }
};

YDEV float be_f32(const uint8_t* q) { uint32_t u = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3]; return __uint_as_float(u); }
YDEV double be_f64(const uint8_t* q) { uint64_t u = 0; for (int i = 0; i < 8; i++) u = (u << 8) | q[i]; return __longlong_as_double((long long)u); }
// lib0 writeAny integer test: 0.2.104 isInteger && abs <= BITS31; 0.2.42 has no abs
YDEV bool js_small_int(double x, uint32_t flags) {
  if (!(x == floor(x)) || isinf(x)) return false;
  if (flags & F_COMPAT_135) return x <= 2147483647.0;
  return fabs(x) <= 2147483647.0;
}

// ---------------------------------------------------------------- Any
// Validates one Any value starting at c.pos (lib0 readAny, L0@4074); *nc set
// when writeAny (L0@8284-8700) would not reproduce the bytes.
template <int D, int K>
YDEV_NI void any_value_t(Cur& c, bool& nc, uint32_t flags) {
  // explicit stack: remaining elements per level; objects alternate key/value
  AnyStack<D, K> st;
  int d = 0;
  const int nm0 = c.nm; c.nm = 0;
  st.rset(0, 1); st.oset(0, 0);
  while (!c.err) {
    if (st.rget(d) == 0) { if (d == 0) break; if (st.oget(d)) st.close_obj(d); d--; continue; }
    st.rset(d, st.rget(d) - 1u);
    if (st.oget(d)) {  // key
      uint32_t kl; const uint32_t ks0 = c.buf(kl);
      if (c.err) break;
      if (utf8_u16(c.p + ks0, kl) < 0) { c.fail(ST_MALFORMED); break; }
      if (kl == 9) { const uint8_t* k = c.p + ks0; if (k[0] == '_' && k[1] == '_' && k[2] == 'p' && k[3] == 'r' && k[4] == 'o' && k[5] == 't' && k[6] == 'o' && k[7] == '_' && k[8] == '_') nc = true; }
      const int kr = st.key(d, c.p + ks0, kl);
      if (kr == 2) { c.fail(ST_FALLBACK); break; }
      if (kr) nc = true;
    }
    const uint8_t tag = c.u8();
    if (c.err) break;
    switch (tag) {
      case 127: case 126: case 121: case 120: break;
      case 125: {  // readVarInt
        const uint8_t r = c.u8(); uint64_t num = r & 63; uint32_t shift = 6;
        if (r & 128) {
          for (;;) {
            const uint8_t b = c.u8(); if (c.err) break;
            if (shift < 60) num |= (uint64_t)(b & 127) << shift; else if (b & 127) { c.fail(ST_RANGE); break; }
            shift += 7;
            if (b < 128) { if (b == 0) nc = true; break; }
            if (num > MAX_SAFE) { c.fail(ST_RANGE); break; }
          }
        }
        if (c.err) break;
        if (num > MAX_SAFE) { c.fail(ST_RANGE); break; }
        if (num > 2147483647ull) nc = true;
        break;
      }
      case 124: {
        if (c.end - c.pos < 4) { c.fail(ST_MALFORMED); break; }
        const float f = be_f32(c.p + c.pos); c.pos += 4;
        if (isnan(f) || js_small_int((double)f, flags)) nc = true;
        break;
      }
      case 123: {
        if (c.end - c.pos < 8) { c.fail(ST_MALFORMED); break; }
        const double x = be_f64(c.p + c.pos); c.pos += 8;
        if (!isnan(x) && (js_small_int(x, flags) || (double)(float)x == x)) nc = true;
        break;
      }
      case 122: if (c.end - c.pos < 8) { c.fail(ST_MALFORMED); break; } c.pos += 8; break;
      case 119: { uint32_t l; const uint32_t s = c.buf(l); if (!c.err && utf8_u16(c.p + s, l) < 0) c.fail(ST_MALFORMED); break; }
      case 116: { uint32_t l; c.buf(l); break; }
      case 117: case 118: {
        const uint64_t n = c.vu();
        if (c.err) break;
        if (d + 1 > D) { c.fail(D == MAX_DEPTH ? ST_DEPTH : ST_FALLBACK); break; }
        if (n > (uint64_t)(c.end - c.pos)) { c.fail(ST_MALFORMED); break; }  // every element takes >= 1 byte
        d++;
        st.rset(d, (uint32_t)n); st.oset(d, tag == 118);
        if (tag == 118) st.open_obj(d);
        break;
      }
      default: c.fail(ST_MALFORMED); break;  // readAnyLookupTable miss -> TypeError
    }
  }
  if (c.nm) nc = true;  // a non-minimal varuint inside the value is re-encoded by writeAny
  c.nm = nm0;
}
YDEV void any_value(Cur& c, bool& nc, uint32_t flags) { any_value_t<MAX_DEPTH, MAX_KEYS>(c, nc, flags); }
// skips one Any value already validated (used to re-walk Any arrays when slicing)
YDEV_NI void any_skip(Cur& c) {
  uint32_t rem[MAX_DEPTH + 1]; uint8_t obj[MAX_DEPTH + 1];
  int d = 0; rem[0] = 1; obj[0] = 0;
  while (!c.err) {
    if (rem[d] == 0) { if (d == 0) break; d--; continue; }
    rem[d]--;
    if (obj[d]) { uint32_t kl; c.buf(kl); }
    const uint8_t tag = c.u8();
    switch (tag) {
      case 125: { uint8_t r = c.u8(); while ((r & 128) && !c.err) r = c.u8(); break; }
      case 124: c.pos += 4; break;
      case 123: case 122: c.pos += 8; break;
      case 119: case 116: { uint32_t l; c.buf(l); break; }
      case 117: case 118: { const uint64_t n = c.vu(); if (d < MAX_DEPTH) { d++; rem[d] = (uint32_t)n; obj[d] = tag == 118; } break; }
      default: break;
    }
  }
}

// ---------------------------------------------------------------- JSON
// JSON.parse grammar + "would JSON.stringify(JSON.parse(s)) === s" (conservative).
// Returns ST_OK / ST_MALFORMED (SyntaxError) / ST_DEPTH; sets nc.
YDEV int hexv(uint8_t ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}
YDEV bool jws(uint8_t ch) { return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r'; }
// parses a JSON string at s[i] == '"'; returns index after closing quote or -1
YDEV_NI int64_t json_string(const uint8_t* s, uint32_t n, uint32_t i, bool& nc, bool& has_esc) {
  i++;
  has_esc = false;
  while (i < n) {
    const uint8_t ch = s[i];
    if (ch == '"') return i + 1;
    if (ch < 0x20) return -1;
    if (ch == '\\') {
      has_esc = true;
      if (i + 1 >= n) return -1;
      const uint8_t e = s[i + 1];
      if (e == '"' || e == '\\' || e == 'b' || e == 'f' || e == 'n' || e == 'r' || e == 't') { i += 2; continue; }
      if (e == '/') { nc = true; i += 2; continue; }
      if (e == 'u') {
        if (i + 6 > n) return -1;
        int v = 0;
        for (int k = 0; k < 4; k++) {
          const int h = hexv(s[i + 2 + k]); if (h < 0) return -1;
          if (s[i + 2 + k] >= 'A' && s[i + 2 + k] <= 'F') nc = true;
          v = v * 16 + h;
        }
        if (!(v < 0x20 && v != 8 && v != 9 && v != 10 && v != 12 && v != 13)) nc = true;
        i += 6; continue;
      }
      return -1;
    }
    i++;
  }
  return -1;
}
// number at s[i]; returns index after or -1.  Canonical (Number::toString) iff:
// no exponent, no "-0"/"0.0", fraction without trailing 0, >= 1e-6 (fewer than
// 6 leading fraction zeros when the integer part is 0), integer part < 22
// digits, <= 15 significant digits.
YDEV_NI int64_t json_number(const uint8_t* s, uint32_t n, uint32_t i, bool& nc) {
  const uint32_t st = i; bool neg = false;
  if (i < n && s[i] == '-') { neg = true; i++; }
  if (i >= n) return -1;
  const uint32_t ib = i;
  if (s[i] == '0') i++;
  else if (s[i] >= '1' && s[i] <= '9') { while (i < n && s[i] >= '0' && s[i] <= '9') i++; }
  else return -1;
  const uint32_t ie = i;
  bool frac = false; uint32_t fb = 0, fe = 0;
  if (i < n && s[i] == '.') {
    i++; fb = i;
    if (i >= n || !(s[i] >= '0' && s[i] <= '9')) return -1;
    while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    fe = i; frac = true;
  }
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    i++;
    if (i < n && (s[i] == '+' || s[i] == '-')) i++;
    if (i >= n || !(s[i] >= '0' && s[i] <= '9')) return -1;
    while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    nc = true;
    return i;
  }
  (void)st;
  const bool int_zero = (ie - ib == 1 && s[ib] == '0');
  if (int_zero) {
    if (!frac) { if (neg) nc = true; return i; }
    // 0.xxx
    uint32_t z = 0; while (fb + z < fe && s[fb + z] == '0') z++;
    if (fb + z == fe) { nc = true; return i; }   // 0.000 == 0
    if (z >= 6) nc = true;                         // < 1e-6 prints with an exponent
    if (s[fe - 1] == '0') nc = true;
    if (fe - fb - z > 15) nc = true;
    return i;
  }
  if (ie - ib >= 22) nc = true;
  int sig;
  if (frac) {
    if (s[fe - 1] == '0') nc = true;
    sig = (int)(ie - ib) + (int)(fe - fb);
  } else {
    uint32_t e = ie; while (e > ib + 1 && s[e - 1] == '0') e--;
    sig = (int)(e - ib);
  }
  if (sig > 15) nc = true;
  return i;
}
template <int D, int K>
YDEV_NI int json_check_t(const uint8_t* s, uint32_t n, bool& nc) {
  // per level: obj (0 array, 1 object, 2 top), state (0 expect value/first, 1 after value, 2 after comma)
  AnyStack<D, K> st;   // (rem holds the state; the top level is d == 0)
  int d = 0;
  uint32_t i = 0;
  // top level: expect exactly one value
  st.oset(0, 0); st.rset(0, 0);
  for (;;) {
    while (i < n && jws(s[i])) { i++; nc = true; }
    const uint32_t lo = d == 0 ? 2u : st.oget(d), ls = st.rget(d);
    if (lo == 2 && ls == 1) { if (i != n) return ST_MALFORMED; return ST_OK; }
    if (ls == 1) {  // after a value inside a container
      if (i >= n) return ST_MALFORMED;
      if (s[i] == ',') { i++; st.rset(d, 2); continue; }
      if ((lo == 1 && s[i] == '}') || (lo == 0 && s[i] == ']')) {
        i++;
        if (lo == 1) st.close_obj(d);
        d--; st.rset(d, 1); continue;
      }
      return ST_MALFORMED;
    }
    if (i >= n) return ST_MALFORMED;
    // state 0 (first element or top) or 2 (after comma)
    if (lo == 1) {
      if (ls == 0 && s[i] == '}') { i++; st.close_obj(d); d--; st.rset(d, 1); continue; }
      if (s[i] != '"') return ST_MALFORMED;
      bool esc; const int64_t e = json_string(s, n, i, nc, esc);
      if (e < 0) return ST_MALFORMED;
      if (esc) nc = true;
      const int kr = st.key(d, s + i + 1, (uint32_t)(e - i - 2));
      if (kr == 2) return ST_FALLBACK;
      if (kr) nc = true;
      i = (uint32_t)e;
      while (i < n && jws(s[i])) { i++; nc = true; }
      if (i >= n || s[i] != ':') return ST_MALFORMED;
      i++;
      while (i < n && jws(s[i])) { i++; nc = true; }
      if (i >= n) return ST_MALFORMED;
    } else if (lo == 0 && ls == 0 && s[i] == ']') { i++; d--; st.rset(d, 1); continue; }
    // a value
    const uint8_t ch = s[i];
    if (ch == '{' || ch == '[') {
      if (d + 1 > D) return D == MAX_DEPTH ? ST_DEPTH : ST_FALLBACK;
      st.rset(d, 1);  // parent resumes after this container
      d++; st.oset(d, ch == '{'); st.rset(d, 0);
      if (ch == '{') st.open_obj(d);
      i++;
      continue;
    }
    int64_t e;
    if (ch == '"') { bool esc; e = json_string(s, n, i, nc, esc); }
    else if (ch == 't') e = (n - i >= 4 && s[i + 1] == 'r' && s[i + 2] == 'u' && s[i + 3] == 'e') ? i + 4 : -1;
    else if (ch == 'f') e = (n - i >= 5 && s[i + 1] == 'a' && s[i + 2] == 'l' && s[i + 3] == 's' && s[i + 4] == 'e') ? i + 5 : -1;
    else if (ch == 'n') e = (n - i >= 4 && s[i + 1] == 'u' && s[i + 2] == 'l' && s[i + 3] == 'l') ? i + 4 : -1;
    else if (ch == '-' || (ch >= '0' && ch <= '9')) e = json_number(s, n, i, nc);
    else e = -1;
    if (e < 0) return ST_MALFORMED;
    i = (uint32_t)e;
    st.rset(d, 1);
  }
}
YDEV int json_check(const uint8_t* s, uint32_t n, bool& nc) { return json_check_t<MAX_DEPTH, MAX_KEYS>(s, n, nc); }

// ---------------------------------------------------------------- structs
// One parsed struct (lazyStructReaderGenerator, Y@36564).
struct SInfo {
  uint8_t kind, info, ref;
  bool nc;           // content would be re-encoded by yjs (non-canonical Any/JSON): refused
  bool renc;         // content holds non-minimal varuints: re-encoded on output (as yjs does)
  uint64_t len;      // clock length
  uint32_t start;    // position of the info byte
  uint32_t cstart;   // position of the content
  uint32_t end;      // position after the struct
};

// readItemContent (Y@81141) validation; returns length in clock units.  SM: the parallel tiers' register stacks for
// Any / JSON nesting (a value past SM_DEPTH levels or SM_KEYS open keys fails the cursor with ST_FALLBACK)
template <bool SM = false>
YDEV_NI uint64_t read_content(Cur& c, uint8_t ref, bool& nc, uint32_t flags) {
  constexpr int D = SM ? SM_DEPTH : MAX_DEPTH, K = SM ? SM_KEYS : MAX_KEYS;
  switch (ref) {
    case 1: return c.vu();                                           // ContentDeleted
    case 2: {                                                        // ContentJSON
      const uint64_t n = c.vu();
      for (uint64_t k = 0; k < n && !c.err; k++) {
        uint32_t l; const uint32_t s = c.buf(l); if (c.err) break;
        if (utf8_u16(c.p + s, l) < 0) { c.fail(ST_MALFORMED); break; }
        const uint8_t* t = c.p + s;
        if (l == 9 && t[0] == 'u' && t[1] == 'n' && t[2] == 'd' && t[3] == 'e' && t[4] == 'f' && t[5] == 'i' && t[6] == 'n' && t[7] == 'e' && t[8] == 'd') continue;
        const int e = json_check_t<D, K>(t, l, nc); if (e) { c.fail(e); break; }
      }
      return n;
    }
    case 3: { uint32_t l; c.buf(l); return 1; }                      // ContentBinary
    case 4: {                                                        // ContentString
      uint32_t l; const uint32_t s = c.buf(l); if (c.err) return 0;
      const int64_t u = utf8_u16(c.p + s, l);
      if (u < 0) { c.fail(ST_MALFORMED); return 0; }
      return (uint64_t)u;
    }
    case 5: {                                                        // ContentEmbed
      uint32_t l; const uint32_t s = c.buf(l); if (c.err) return 1;
      if (utf8_u16(c.p + s, l) < 0) { c.fail(ST_MALFORMED); return 1; }
      const int e = json_check_t<D, K>(c.p + s, l, nc); if (e) c.fail(e);
      return 1;
    }
    case 6: {                                                        // ContentFormat
      uint32_t l; uint32_t s = c.buf(l); if (c.err) return 1;
      if (utf8_u16(c.p + s, l) < 0) { c.fail(ST_MALFORMED); return 1; }
      s = c.buf(l); if (c.err) return 1;
      if (utf8_u16(c.p + s, l) < 0) { c.fail(ST_MALFORMED); return 1; }
      const int e = json_check_t<D, K>(c.p + s, l, nc); if (e) c.fail(e);
      return 1;
    }
    case 7: {                                                        // ContentType
      const uint64_t tr = c.vu(); if (c.err) return 1;
      if (tr > 6) { c.fail(ST_MALFORMED); return 1; }
      if (tr == 3 || tr == 5) { uint32_t l; const uint32_t s = c.buf(l); if (!c.err && utf8_u16(c.p + s, l) < 0) c.fail(ST_MALFORMED); }
      return 1;
    }
    case 8: {                                                        // ContentAny
      const uint64_t n = c.vu();
      for (uint64_t k = 0; k < n && !c.err; k++) any_value_t<D, K>(c, nc, flags);
      return n;
    }
    case 9: {                                                        // ContentDoc (Y@70773)
      uint32_t l; const uint32_t s = c.buf(l); if (c.err) return 1;
      if (utf8_u16(c.p + s, l) < 0) { c.fail(ST_MALFORMED); return 1; }
      const uint32_t o0 = c.pos;
      bool anc = false; any_value_t<D, K>(c, anc, flags);
      if (c.err) return 1;
      if (anc) nc = true;
      // canonical iff an object whose keys are an ordered subset of gc:false, autoLoad:true, meta:<non-null>
      Cur q{c.p, o0, c.pos, 0, 0};
      if (q.u8() != 118) { nc = true; return 1; }
      const uint64_t nk = q.vu(); int stage = 0;
      for (uint64_t k = 0; k < nk && !q.err; k++) {
        uint32_t kl; const uint32_t ks = q.buf(kl);
        const uint8_t* key = q.p + ks; const uint8_t vt = q.p[q.pos];
        bool vnc = false; any_value_t<D, K>(q, vnc, flags);
        if (kl == 2 && key[0] == 'g' && key[1] == 'c' && stage < 1 && vt == 121) stage = 1;
        else if (kl == 8 && key[0] == 'a' && key[1] == 'u' && key[2] == 't' && key[3] == 'o' && key[4] == 'L' && key[5] == 'o' && key[6] == 'a' && key[7] == 'd' && stage < 2 && vt == 120) stage = 2;
        else if (kl == 4 && key[0] == 'm' && key[1] == 'e' && key[2] == 't' && key[3] == 'a' && stage < 3 && vt != 126 && vt != 127 && !vnc) stage = 3;
        else nc = true;
      }
      return 1;
    }
    default: c.fail(ST_MALFORMED); return 0;  // contentRefs[0] / [10] -> unexpectedCase; > 10 TypeError
  }
}

// Parses the struct at c.pos.  Header varuints are re-encoded on output, so
// only content varuints count toward `nc`.
template <bool SM = false>
YDEV_NI void read_struct(Cur& c, SInfo& s, uint32_t flags) {
  s.start = c.pos; s.nc = false; s.renc = false; s.ref = 0;
  const uint8_t info = c.u8();
  s.info = info;
  if (c.err) return;
  if (info == 10) { s.kind = K_SKIP; s.len = c.vu(); s.cstart = c.pos; s.end = c.pos; return; }
  if ((info & 31) == 0) { s.kind = K_GC; s.len = c.vu(); s.cstart = c.pos; s.end = c.pos; return; }
  s.kind = K_ITEM; s.ref = info & 31;
  if (info & 0x80) { c.vu(); c.vu(); }
  if (info & 0x40) { c.vu(); c.vu(); }
  if ((info & 0xC0) == 0) {
    const uint64_t pi = c.vu();
    if (pi == 1) { uint32_t l; const uint32_t s0 = c.buf(l); if (!c.err && utf8_u16(c.p + s0, l) < 0) c.fail(ST_MALFORMED); }
    else { c.vu(); c.vu(); }
    if (info & 0x20) { uint32_t l; const uint32_t s0 = c.buf(l); if (!c.err && utf8_u16(c.p + s0, l) < 0) c.fail(ST_MALFORMED); }
  }
  if (c.err) return;
  s.cstart = c.pos;
  if (s.ref == 10) { c.fail(ST_MALFORMED); return; }
  const int nm0 = c.nm; c.nm = 0;
  bool nc = false;
  s.len = read_content<SM>(c, s.ref, nc, flags);
  if (c.nm) s.renc = true;  // Any values track their own non-minimal varuints (-> nc)
  c.nm = nm0;
  s.nc = nc;
  s.end = c.pos;
}

// read_struct for a cursor that must stay in registers: the shapes of text logs (Skip, GC, an Item with origin(s)
// and ContentDeleted / ContentString) are read inline with exactly read_struct's reads and results; anything else
// goes to read_struct through a copy of the cursor (a cursor whose address reaches a non-inlined call lives in
// scratch memory for the whole function: one scratch round trip per byte read).
template <bool SM = false>
YDEV void read_struct_fast(Cur& c, SInfo& s, uint32_t flags) {
  const uint32_t p0 = c.pos;
  if (c.pos < c.end) {
    const uint8_t info = c.p[c.pos];
    const uint8_t ref = info & 31;
    if (info == 10 || ref == 0) {   // Skip / GC: a varuint length
      c.pos++;
      s.start = p0; s.nc = false; s.renc = false; s.ref = 0; s.info = info;
      s.kind = info == 10 ? K_SKIP : K_GC; s.len = c.vu(); s.cstart = c.pos; s.end = c.pos;
      return;
    }
    if ((info & 0xC0) && (ref == 1 || ref == 4)) {
      c.pos++;
      s.start = p0; s.nc = false; s.renc = false; s.info = info; s.kind = K_ITEM; s.ref = ref;
      if (info & 0x80) { c.vu(); c.vu(); }
      if (info & 0x40) { c.vu(); c.vu(); }
      if (c.err) return;
      s.cstart = c.pos;
      const int nm0 = c.nm; c.nm = 0;
      if (ref == 1) s.len = c.vu();
      else {
        uint32_t l; const uint32_t st = c.buf(l);
        s.len = 0;
        if (!c.err) {
          bool ascii = true;
          for (uint32_t i = 0; i < l; i++) ascii = ascii && c.p[st + i] < 0x80;
          const int64_t u = ascii ? (int64_t)l : utf8_u16(c.p + st, l);
          if (u < 0) c.fail(ST_MALFORMED); else s.len = (uint64_t)u;
        }
      }
      if (c.nm) s.renc = true;
      c.nm = nm0;
      s.end = c.pos;
      return;
    }
  }
  Cur t = c;
  read_struct<SM>(t, s, flags);
  c = t;
}

// ---------------------------------------------------------------- writers
// Output sink: a plain byte pointer (global memory or LDS).  All writers
// return the number of bytes and, when `o` is non-null, store them.
struct Out {
  uint8_t* p; uint32_t n;
  YDEV void b(uint8_t v) { if (p) p[n] = v; n++; }
  YDEV void vu(uint64_t v) { while (v > 127) { b((uint8_t)(0x80 | (v & 127))); v >>= 7; } b((uint8_t)v); }
  YDEV void copy(const uint8_t* s, uint32_t len) { if (p) for (uint32_t i = 0; i < len; i++) p[n + i] = s[i]; n += len; }
};

// UTF-16 offset -> byte offset in UTF-8; *mid when the cut splits a surrogate pair
YDEV uint32_t u16_to_byte(const uint8_t* s, uint32_t n, uint64_t off, bool& mid) {
  uint32_t i = 0; uint64_t u = 0; mid = false;
  while (i < n && u < off) {
    const uint8_t ch = s[i];
    const uint32_t k = ch < 0x80 ? 1 : (ch & 0xE0) == 0xC0 ? 2 : (ch & 0xF0) == 0xE0 ? 3 : 4;
    if (k == 4) { if (u + 1 == off) { mid = true; return i + 4; } u += 2; }
    else u += 1;
    i += k;
  }
  return i;
}

// Writes an item's content with `off` leading clock units removed
// (ContentX.write(encoder, offset) / ContentX.splice, Y@69266-73441).
// `splice` selects sliceStruct's splice (always U+FFFD) over write(offset)
// (U+FFFD in 13.6 / throw in 13.5 compat).  Returns ST_OK or an error.
YDEV_NI int write_content(Out& o, const uint8_t* base, const SInfo& s, uint64_t off, bool splice, uint32_t flags) {
  Cur c{base, s.cstart, s.end, 0, 0};
  if (off == 0 && !s.renc) { o.copy(base + s.cstart, s.end - s.cstart); return ST_OK; }
  switch (s.ref) {
    case 1: { const uint64_t n = c.vu(); o.vu(n - off); return ST_OK; }
    case 2: case 8: {
      const uint64_t n = c.vu();
      o.vu(n - off);
      for (uint64_t k = 0; k < n && !c.err; k++) {
        const uint32_t a = c.pos;
        if (s.ref == 2) {
          uint32_t l; const uint32_t st = c.buf(l);
          if (k >= off) { o.vu(l); o.copy(base + st, l); }
        } else {
          any_skip(c);
          if (k >= off) o.copy(base + a, c.pos - a);
        }
      }
      return ST_OK;
    }
    case 4: {
      uint32_t l; const uint32_t st = c.buf(l);
      bool mid; const uint32_t b = off ? u16_to_byte(base + st, l, off, mid) : (mid = false, 0u);
      if (mid) {
        if (!splice && (flags & F_COMPAT_135)) return ST_SURROGATE;
        o.vu((uint64_t)(l - b) + 3); o.b(0xEF); o.b(0xBF); o.b(0xBD);
      } else o.vu(l - b);
      o.copy(base + st + b, l - b);
      return ST_OK;
    }
    case 3: case 5: { uint32_t l; const uint32_t st = c.buf(l); o.vu(l); o.copy(base + st, l); return ST_OK; }
    case 6: {
      uint32_t l; uint32_t st = c.buf(l); o.vu(l); o.copy(base + st, l);
      st = c.buf(l); o.vu(l); o.copy(base + st, l);
      return ST_OK;
    }
    case 7: {
      const uint64_t tr = c.vu(); o.vu(tr);
      if (tr == 3 || tr == 5) { uint32_t l; const uint32_t st = c.buf(l); o.vu(l); o.copy(base + st, l); }
      return ST_OK;
    }
    case 9: {
      uint32_t l; const uint32_t st = c.buf(l); o.vu(l); o.copy(base + st, l);
      o.copy(base + c.pos, s.end - c.pos);
      return ST_OK;
    }
    default: return ST_MALFORMED;
  }
}

// Item.write(encoder, offset) (Y@80416) re-encoding the header from the input
// struct; GC/Skip write (Y@68955/Y@81211).  `off` > 0 makes origin =
// (client, clock+off-1).  Returns ST_OK or error.
YDEV_NI int write_struct(Out& o, const uint8_t* base, const SInfo& s, uint64_t client, uint64_t clock, uint64_t off,
                      bool splice, uint32_t flags) {
  if (s.kind == K_GC) { o.b(0); o.vu(s.len - off); return ST_OK; }
  if (s.kind == K_SKIP) { o.b(10); o.vu(s.len - off); return ST_OK; }
  if (s.nc) return ST_NONCANON;
  Cur c{base, s.start + 1, s.cstart, 0, 0};
  const uint8_t info = s.info;
  const bool ho = (info & 0x80) != 0, hr = (info & 0x40) != 0;
  uint64_t oc = 0, ok = 0, rc = 0, rk = 0;
  if (ho) { oc = c.vu(); ok = c.vu(); }
  if (hr) { rc = c.vu(); rk = c.vu(); }
  const bool has_sub = !ho && !hr && (info & 0x20);  // parentSub only read without origins
  const bool o_out = ho || off > 0;
  if (off > 0) { oc = client; ok = clock + off - 1; }
  const bool sub_bit = has_sub || ((flags & F_KEEP_SUB) && (info & 0x20));
  o.b((uint8_t)((info & 31) | (o_out ? 0x80 : 0) | (hr ? 0x40 : 0) | (sub_bit ? 0x20 : 0)));
  if (o_out) { o.vu(oc); o.vu(ok); }
  if (hr) { o.vu(rc); o.vu(rk); }
  if (!ho && !hr) {
    const uint64_t pi = c.vu();
    uint32_t pkl = 0, pks = 0; uint64_t pc = 0, pk = 0;
    if (pi == 1) pks = c.buf(pkl); else { pc = c.vu(); pk = c.vu(); }
    uint32_t sl = 0, ss = 0;
    if (info & 0x20) ss = c.buf(sl);
    if (!o_out) {  // parent written only when neither origin is set
      if (pi == 1) { o.b(1); o.vu(pkl); o.copy(base + pks, pkl); }
      else { o.b(0); o.vu(pc); o.vu(pk); }
      if (has_sub) { o.vu(sl); o.copy(base + ss, sl); }
    }
  }
  return write_content(o, base, s, off, splice, flags);
}

}  // namespace ygm
