// ygm_merge_wave.hpp -- mergeUpdates for small documents: ONE WAVE (64 lanes) PER DOCUMENT.
//
// The common Hocuspocus shape (a snapshot plus ~200
// single-transaction updates, a few KB per document) is far too small for a
// workgroup, so each wave owns one document end to end with no workgroup
// barriers:
//   stage    16-byte loads of the document's bytes into the wave's LDS slice
//   parse    ONE pass, lane per update (strided); varuints decoded branch-free from an
//            unaligned 8-byte LDS window; struct records get wave-aggregated slots
//   clients  distinct clients by wave vote (<= 64), ranked descending
//   sort     in-register bitonic sort of (client rank, clock, record) keys, 1-4 per lane
//   scan     rule R-M: Skip gaps, provenance-dependent GC coalescing,
//            block struct counts; rule R-DS for the delete set -- wave shuffles only
//   emit     lane-contiguous segments into an LDS output buffer, then coalesced 16-byte
//            stores into the document's own 16-byte aligned output slot
// Documents over the caps are deferred to the workgroup kernel (k_merge_fast).
#pragma once
#include "ygm_common.hpp"

namespace ygm {

constexpr int W_WAVES = 1;     // documents per workgroup (one wave each: LDS-granular occupancy)
constexpr int W_K = 256;       // updates
constexpr int W_IN = 8192;     // staged input bytes (realistic 200-update logs of multi-character inserts: ~6 KB)
constexpr int W_OUT = 8192;    // staged output bytes
constexpr int W_S = 256;       // non-Skip structs
constexpr int W_D = 128;       // delete-set ranges
constexpr int W_C = 64;        // distinct clients in the struct section
constexpr int W_E = W_S / WAVE;
constexpr int W_DE = W_D / WAVE;
constexpr int W_BLK = 64;      // delete-set clients

struct alignas(16) WaveLds {
  uint8_t in[W_IN + 16];     // staged bytes (+ slack: window reads reach end + 15)
  uint8_t out[W_OUT];        // staged output (16-byte aligned)
  union {
    struct { uint16_t ustart[W_K], ulen[W_K]; };   // parse
    struct {                                       // after the sort
      uint8_t eflag[W_S];    // per sorted element: EF_* bits
      uint16_t epos[W_S];    // per sorted element: output offset inside the struct section
      uint32_t blkcnt[W_C];  // structs per client block
    };
  };
  uint64_t key[W_S];         // by record: clock << 8 | record; then sorted keys (client rank << 40 | ...)
  uint64_t ra[W_S];          // by record: start << 48 | byte length << 32 | clock length
  uint32_t rb[W_S];          // by record: (update << 8 | seq) << 16 | kind/slow << 13 | re-encoded length
  uint32_t rcl[W_S];         // by record: client; after the sort: GC run end by sorted element
  uint32_t ctab[W_C];        // clients by rank (descending)
  uint64_t dkey[W_D];        // permuted in place into rank order
  uint32_t dlen[W_D];
  uint8_t dflag[W_D];        // bit 0 segment start, bit 1 run start, bits 2-7 segment id
  uint16_t dposs[W_D];
  uint32_t segcnt[W_BLK];
  uint32_t drunend[W_D];     // (the parse parks each record's first-seen rank here: yjs 13.5's client order)
  uint32_t dcl[W_D];         // by record, then permuted with dkey: client
  uint32_t nrec, ndel;
};

// LDS-typed views: keep ds_* addressing across non-inlined helpers
typedef __attribute__((address_space(3))) WaveLds LWave;
typedef __attribute__((address_space(3))) const uint8_t LU8;
typedef __attribute__((address_space(3))) const uint64_t LU64;

YDEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Literal lib0 readVarUint over LDS bytes (Cur::vu semantics) for varuints the
// window decoder does not take (> 8 bytes or running past the end).  Free
// function, results by value: the reader itself stays in registers.
struct VuRes { uint64_t v; uint32_t pos; int err, nm; };
YDEV_NI VuRes vu_slow(LU8* base, uint32_t pos, uint32_t end) {
  uint64_t num = 0; uint32_t shift = 0;
  for (;;) {
    if (pos >= end) return VuRes{0, end, ST_MALFORMED, 0};
    const uint8_t r = base[pos++];
    if (shift < 63) num |= (uint64_t)(r & 127) << shift;
    else if (r & 127) return VuRes{0, end, ST_RANGE, 0};
    shift += 7;
    if (r < 128) {
      if (num > MAX_SAFE) return VuRes{0, end, ST_RANGE, 0};
      return VuRes{num, pos, 0, (r == 0 && shift > 7) ? 1 : 0};
    }
    if (num > MAX_SAFE) return VuRes{0, end, ST_RANGE, 0};
  }
}

// Reader over the staged LDS bytes.  peek8() = the 8 bytes at pos from two
// aligned ds_read_b64; vu() decodes a varuint of <= 8 bytes without a byte
// loop (terminator by bit trick, 7-bit groups gathered by three mask/shift
// steps) and takes the literal loop (Cur::vu semantics) otherwise.
struct WinRd {
  LU8* base;
  uint32_t pos, end;
  int err, nm;
  YDEV void init(LU8* b, uint32_t p, uint32_t e) { base = b; pos = p; end = e; err = 0; nm = 0; }
  YDEV void fail(int e) { if (!err) err = e; pos = end; }
  YDEV const uint8_t* generic() const { return (const uint8_t*)base; }
  YDEV uint64_t peek8() const {
    const uint32_t a = pos & ~7u, sh = (pos & 7u) * 8u;
    const uint64_t lo = *(LU64*)(base + a), hi = *(LU64*)(base + a + 8);
    return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
  }
  YDEV uint8_t u8() {
    if (pos >= end) { fail(ST_MALFORMED); return 0; }
    return base[pos++];
  }
  YDEV uint64_t vu() {
    const uint64_t w = peek8();
    const uint64_t t = ~w & 0x8080808080808080ull;
    const uint32_t n = t ? (uint32_t)(__builtin_ctzll(t) >> 3) + 1u : 9u;
    if (n > 8 || pos + n > end) {
      const VuRes v = vu_slow(base, pos, end);
      pos = v.pos; nm |= v.nm;
      if (v.err) fail(v.err);
      return v.v;
    }
    uint64_t x = (n == 8 ? w : (w & ((1ull << (8u * n)) - 1ull))) & 0x7f7f7f7f7f7f7f7full;
    x = ((x >> 1) & 0x3f803f803f803f80ull) | (x & 0x007f007f007f007full);
    x = ((x >> 2) & 0x0fffc0000fffc000ull) | (x & 0x00003fff00003fffull);
    x = ((x >> 4) & 0x00fffffff0000000ull) | (x & 0x000000000fffffffull);
    if (x > MAX_SAFE) { fail(ST_RANGE); return 0; }
    if (n > 1 && (uint8_t)(w >> (8u * (n - 1u))) == 0) nm = 1;
    pos += n;
    return x;
  }
  // skips n bytes that must be 7-bit ASCII; false if any is not (-> general parser)
  YDEV bool ascii(uint64_t n) {
    if (n > (uint64_t)(end - pos)) { fail(ST_MALFORMED); return true; }
    uint32_t left = (uint32_t)n;
    bool ok = true;
    while (left) {
      const uint32_t m = left < 8u ? left : 8u;
      const uint64_t w = peek8() & (m == 8 ? ~0ull : ((1ull << (8u * m)) - 1ull));
      ok &= (w & 0x8080808080808080ull) == 0;
      pos += m; left -= m;
    }
    return ok;
  }
};

// Parses one struct at r.pos.  Fast inline path for GC / Skip / Items with
// Deleted or ASCII String content and ASCII parent keys; everything else goes
// through the general validator (read_struct).  Returns the kind, clock length,
// byte length of the re-encoded struct (out_len) and whether it must be
// re-encoded on output (slow) or is non-canonical (nc).
YDEV void w_struct(WinRd& r, uint32_t flags, uint8_t& kind, uint64_t& len, uint32_t& out_len, bool& slow, bool& nc) {
  const uint32_t start = r.pos;
  const int nm0 = r.nm; r.nm = 0;
  slow = false; nc = false; out_len = 0; len = 0;
  const uint8_t info = r.u8();
  if (r.err) return;
  if (info == 10) { kind = K_SKIP; len = r.vu(); r.nm = nm0; return; }
  if ((info & 31) == 0) { kind = K_GC; len = r.vu(); r.nm = nm0; return; }
  kind = K_ITEM;
  const uint8_t ref = info & 31;
  bool fast = ref == 1 || ref == 4;
  if (fast) {
    if (info & 0x80) { r.vu(); r.vu(); }
    if (info & 0x40) { r.vu(); r.vu(); }
    if ((info & 0xC0) == 0) {
      const uint64_t pi = r.vu();
      if (pi > 1) r.nm = 1;  // parentInfo is written back as 0 (non-key): re-encode
      if (pi == 1) { const uint64_t l = r.vu(); if (!r.err && !r.ascii(l)) fast = false; }
      else { r.vu(); r.vu(); }
      if (fast && (info & 0x20)) { const uint64_t l = r.vu(); if (!r.err && !r.ascii(l)) fast = false; }
    }
    if (fast && !r.err) {
      len = r.vu();
      if (ref == 4 && !r.err && !r.ascii(len)) fast = false;
    }
  }
  if (r.err) { r.nm = nm0; return; }
  if (fast) {
    out_len = r.pos - start;
    slow = r.nm != 0;  // a non-minimal varuint / parentInfo: the writer re-encodes (different length)
    if (slow) {
      Out o{nullptr, 0}; Cur c{r.generic(), start, r.end, 0, 0}; SInfo si; read_struct<true>(c, si, flags);
      if (c.err) { r.fail(c.err); r.nm = nm0; return; }
      write_struct(o, r.generic(), si, 0, 0, 0, false, flags); out_len = o.n;
    }
    r.nm = nm0;
    return;
  }
  // general path (noinline validator over a generic pointer)
  Cur c{r.generic(), start, r.end, 0, 0};
  SInfo si; read_struct<true>(c, si, flags);
  if (c.err) { r.fail(c.err); return; }
  r.pos = c.pos;
  len = si.len; nc = si.nc;
  Out o{nullptr, 0};
  slow = true;  // general-path items are always written by write_struct
  if (!si.nc) write_struct(o, r.generic(), si, 0, 0, 0, false, flags);
  out_len = o.n;
  r.nm = nm0;
}

// dword-combining global writer for one lane's contiguous output segment
struct GWriter {
  uint8_t* out; uint64_t pos, seg_start; uint32_t acc;
  YDEV void init(uint8_t* o, uint64_t p) { out = o; pos = p; seg_start = p; acc = 0; }
  YDEV void b(uint8_t v) {
    const uint32_t sh = (uint32_t)(pos & 3u) * 8u;
    acc |= (uint32_t)v << sh;
    if ((pos & 3u) == 3u) {
      const uint64_t ws = pos & ~3ull;
      if (ws >= seg_start) *(uint32_t*)(out + ws) = acc;        // whole word is this lane's
      else for (uint64_t q = seg_start; q <= pos; q++) out[q] = (uint8_t)(acc >> ((q & 3u) * 8u));
      acc = 0;
    }
    pos++;
  }
  YDEV void vu(uint64_t v) { while (v > 127) { b((uint8_t)(0x80 | (v & 127))); v >>= 7; } b((uint8_t)v); }
  YDEV void flush() {  // partial trailing word: byte stores (neighbouring lanes own the rest)
    if (pos & 3u) {
      const uint64_t ws = pos & ~3ull;
      const uint64_t from = ws > seg_start ? ws : seg_start;
      for (uint64_t q = from; q < pos; q++) out[q] = (uint8_t)(acc >> ((q & 3u) * 8u));
    }
    acc = 0;
  }
  // n bytes were written at pos by someone else (after a flush()): skip them
  YDEV void jump(uint64_t n) { pos += n; seg_start = pos; acc = 0; }
};

// LDS output writer for one lane's contiguous segment (byte stores; segments are disjoint)
typedef __attribute__((address_space(3))) uint8_t LO8;
struct LWriter {
  LO8* o; uint32_t pos;
  YDEV void b(uint8_t v) { o[pos++] = v; }
  YDEV void vu(uint32_t v) { while (v > 127) { o[pos++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[pos++] = (uint8_t)v; }
  // n bytes from the staged input at s: one 8-byte window read per 8 bytes
  YDEV void copy(LU8* in, uint32_t s, uint32_t n) {
    while (n) {
      const uint32_t a = s & ~7u, sh = (s & 7u) * 8u;
      const uint64_t lo = *(LU64*)(in + a), hi = *(LU64*)(in + a + 8);
      const uint64_t w = sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
      const uint32_t m = n < 8u ? n : 8u;
#pragma unroll
      for (uint32_t i = 0; i < 8; i++) if (i < m) o[pos + i] = (uint8_t)(w >> (8u * i));
      pos += m; s += m; n -= m;
    }
  }
};

YDEV uint32_t wave_exscan(uint32_t v, uint32_t& total) {
  const uint32_t inc = wave_incl_scan_add(v);
  total = __shfl(inc, WAVE - 1, WAVE);
  return inc - v;
}

// slot for the calling lane among the currently active lanes (one LDS atomic per wave)
YDEV uint32_t wave_slot(__attribute__((address_space(3))) uint32_t* ctr) {
  const uint64_t m = __ballot(1);
  const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1u;
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  uint32_t base = 0;
  if (lane_id() == leader) base = atomicAdd((uint32_t*)ctr, (uint32_t)__popcll(m));
  return (uint32_t)__shfl((int)base, (int)leader, WAVE) + rank;
}

struct UpdCount { int err; uint32_t fb, nc; };

// The single parse pass over update i: validates every byte (yjs reads all of
// them), writes struct records (slot from the wave counter L->nrec) and
// delete-set ranges (L->ndel).  One non-inlined instance.
YDEV UpdCount w_parse_update(LWave* L, int i, uint32_t flags) {
  WinRd r; r.init(L->in, L->ustart[i], (uint32_t)L->ustart[i] + L->ulen[i]);
  bool fb = false, nc = false;
  uint64_t prev_client = 0, prev_end = 0; bool have_prev = false;
  uint32_t seq = 0;
  const uint64_t nb = r.vu();
  for (uint64_t b = 0; b < nb && !r.err; b++) {
    const uint64_t nst = r.vu(), client = r.vu(); uint64_t clock = r.vu();
    if (r.err) break;
    if (client > 0xFFFFFFFFull) fb = true;
    for (uint64_t s = 0; s < nst && !r.err; s++) {
      const uint32_t start = r.pos;
      uint8_t kind; uint64_t len; uint32_t olen; bool slow, snc;
      w_struct(r, flags, kind, len, olen, slow, snc);
      if (r.err) break;
      const uint64_t end = clock + len;
      if (end > MAX_SAFE) { r.fail(ST_RANGE); break; }
      if (kind != K_SKIP) {
        if (len == 0 || end > 0xFFFFFFFFull || olen > 0x1FFFu || seq > 255) fb = true;
        if (have_prev && (client > prev_client || (client == prev_client && clock < prev_end))) fb = true;
        have_prev = true; prev_client = client; prev_end = end;
        if (snc) nc = true;
        if (!fb) {
          const uint32_t j = wave_slot(&L->nrec);
          if (j < (uint32_t)W_S) {
            L->key[j] = ((uint64_t)(uint32_t)clock << 8) | j;
            L->ra[j] = ((uint64_t)start << 48) | ((uint64_t)(r.pos - start) << 32) | (uint32_t)len;
            L->rb[j] = ((uint32_t)((i << 8) | seq) << 16) | ((uint32_t)(kind | (slow ? 4 : 0)) << 13) | olen;
            L->rcl[j] = (uint32_t)client;
          }
        }
        seq++;
      }
      clock = end;
    }
  }
  const uint64_t ncl = r.err ? 0 : r.vu();
  uint32_t rr = 0;   // ranges of this update so far: (update << 8 | rr) is the range's first-seen rank
  for (uint64_t q = 0; q < ncl && !r.err; q++) {
    const uint64_t cl = r.vu(), nr = r.vu();
    for (uint64_t k = 0; k < nr && !r.err; k++) {
      const uint64_t ck = r.vu(), ln = r.vu();
      if (r.err) break;
      if (cl > 0xFFFFFFFFull || ck + ln > 0xFFFFFFFFull) fb = true;
      if (!fb) {
        const uint32_t j = wave_slot(&L->ndel);
        if (j < (uint32_t)W_D) {
          L->dkey[j] = ((uint64_t)(0xFFFFFFFFu - (uint32_t)cl) << 32) | (uint32_t)ck; L->dlen[j] = (uint32_t)ln;
          L->dcl[j] = (uint32_t)cl; L->drunend[j] = ((uint32_t)i << 8) | (rr < 255u ? rr : 255u);
        }
      }
      rr++;
    }
  }
  return UpdCount{r.err, fb ? 1u : 0u, nc ? 1u : 0u};
}

// In-register bitonic sort (ascending) of 64*E keys; lane l holds elements E*l .. E*l+E-1.
template <int E>
YDEV void wave_bitonic(uint64_t (&k)[4]) {
  const uint32_t l = lane_id();
  constexpr uint32_t N = 64u * E;
  for (uint32_t kk = 2; kk <= N; kk <<= 1) {
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      if (j >= (uint32_t)E) {  // partner in lane l ^ (j / E), same register
        const int lx = (int)(j / E);
#pragma unroll
        for (int q = 0; q < E; q++) {
          const uint64_t p = __shfl_xor(k[q], lx, WAVE);
          const uint32_t i = E * l + q;
          const bool keep_min = ((i & j) == 0) == ((i & kk) == 0);
          const uint64_t mn = p < k[q] ? p : k[q], mx = p < k[q] ? k[q] : p;
          k[q] = keep_min ? mn : mx;
        }
      } else if (j == 1) {     // pairs (0,1), (2,3) inside the lane
#pragma unroll
        for (int q = 0; q + 1 < E; q += 2) {
          const bool a = ((E * l + q) & kk) == 0;
          const uint64_t x = k[q], y = k[q + 1];
          const uint64_t mn = x < y ? x : y, mx = x < y ? y : x;
          k[q] = a ? mn : mx; k[q + 1] = a ? mx : mn;
        }
      } else {                 // j == 2, E == 4: pairs (0,2), (1,3)
#pragma unroll
        for (int q = 0; q < 2 && E == 4; q++) {
          const bool a = ((E * l + q) & kk) == 0;
          const uint64_t x = k[q], y = k[q + 2];
          const uint64_t mn = x < y ? x : y, mx = x < y ? y : x;
          k[q] = a ? mn : mx; k[q + 2] = a ? mx : mn;
        }
      }
    }
  }
}

}  // namespace ygm
