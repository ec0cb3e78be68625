// ygm_merge_wave.hpp -- mergeUpdates for small documents: ONE WAVE (64 lanes) PER DOCUMENT.
//
// The common Hocuspocus shape (a snapshot plus ~200
// single-transaction updates, a few KB per document) is far too small for a
// workgroup, so each wave owns one document end to end with no workgroup
// barriers:
//   stage    16-byte coalesced loads of the document's bytes into the wave's LDS slice
//   parse    lane per update (blocked), through an 8-byte-window LDS reader
//   sort     rank sort of (client desc, clock asc) keys (S <= 256: each lane ranks its
//            4 keys against all S with broadcast LDS reads; ties -> overlap -> sequential kernel)
//   scan     rule R-M: Skip gaps, provenance-dependent GC coalescing,
//            block struct counts; rule R-DS for the delete set -- wave shuffles only
//   emit     lane-contiguous output segments through a dword-combining writer
// Documents over the caps are deferred to the workgroup kernel (k_merge_fast).
#pragma once
#include "ygm_common.hpp"

namespace ygm {

constexpr int W_WAVES = 2;     // documents per workgroup (one per wave)
constexpr int W_K = 256;       // updates
constexpr int W_IN = 6144;     // staged input bytes
constexpr int W_S = 256;       // non-Skip structs
constexpr int W_D = 128;       // delete-set ranges
constexpr int W_R = W_K / WAVE;
constexpr int W_E = W_S / WAVE;
constexpr int W_DE = W_D / WAVE;
constexpr int W_BLK = 64;      // client blocks (struct section) and delete-set clients

struct WaveLds {
  uint8_t in[W_IN + 32];
  uint16_t ustart[W_K], ulen[W_K];
  uint16_t uns[W_K], und[W_K];   // per-update struct / delete-range counts (pass A)
  uint64_t key[W_S];         // by record id; permuted in place into rank order by the sort
  uint16_t sidx[W_S];        // rank -> record id
  uint16_t r_start[W_S], r_blen[W_S], r_ss[W_S];
  uint32_t r_len[W_S];
  uint8_t r_flag[W_S];       // bits 0-1 kind, bit 2 slow-emit
  uint16_t r_out[W_S];       // re-encoded byte length of an item
  uint8_t eflag[W_S];        // per sorted element: EF_* bits
  uint8_t eblk[W_S];         // per sorted element: client-block index (< W_BLK)
  uint16_t epos[W_S];        // per sorted element: output offset inside the struct section
  uint8_t dflag[W_D], dsid[W_D];
  uint16_t dposs[W_D];
  uint32_t blkcnt[W_BLK];
  uint32_t runend[W_S];
  uint64_t dkey[W_D];        // permuted in place into rank order
  uint32_t dlen[W_D];
  uint32_t segcnt[W_BLK];
  uint32_t drunend[W_D];
};

// LDS-typed views: keep ds_* addressing across non-inlined helpers
typedef __attribute__((address_space(3))) WaveLds LWave;
typedef __attribute__((address_space(3))) const uint8_t LU8;

YDEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Byte reader over an 8-byte-aligned LDS buffer: one ds_read_b64 per 8 bytes.
struct WinRd {
  LU8* base;
  uint32_t pos, end, wat;
  uint64_t win;
  int err, nm;
  YDEV void init(LU8* b, uint32_t p, uint32_t e) { base = b; pos = p; end = e; wat = 0xFFFFFFFFu; win = 0; err = 0; nm = 0; }
  YDEV void fail(int e) { if (!err) err = e; pos = end; }
  YDEV const uint8_t* generic() const { return (const uint8_t*)base; }
  YDEV uint8_t u8() {
    if (pos >= end) { fail(ST_MALFORMED); return 0; }
    const uint32_t a = pos & ~7u;
    if (a != wat) { wat = a; win = *(__attribute__((address_space(3))) const uint64_t*)(base + a); }
    const uint8_t v = (uint8_t)(win >> ((pos & 7u) * 8u));
    pos++;
    return v;
  }
  YDEV uint64_t vu() {
    uint64_t num = 0; uint32_t shift = 0;
    for (;;) {
      if (pos >= end) { fail(ST_MALFORMED); return 0; }
      const uint8_t r = u8();
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
  // skips n bytes that must be 7-bit ASCII; false if any is not (-> general parser)
  YDEV bool ascii(uint64_t n) {
    if (n > (uint64_t)(end - pos)) { fail(ST_MALFORMED); return true; }
    for (uint32_t i = 0; i < (uint32_t)n; i++) if (u8() & 0x80) return false;
    return true;
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
  slow = false; nc = false;
  const uint8_t info = r.u8();
  if (r.err) return;
  if (info == 10) { kind = K_SKIP; len = r.vu(); out_len = 0; r.nm = nm0; return; }
  if ((info & 31) == 0) { kind = K_GC; len = r.vu(); out_len = 0; r.nm = nm0; return; }
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
      if (ref == 1) len = r.vu();
      else { len = r.vu(); if (!r.err && !r.ascii(len)) fast = false; }
    }
  }
  if (r.err) { r.nm = nm0; return; }
  if (fast) {
    out_len = r.pos - start;
    slow = r.nm != 0;  // a non-minimal varuint: the writer re-encodes (different length)
    if (slow) { Out o{nullptr, 0}; Cur c{r.generic(), start, r.end, 0, 0}; SInfo si; read_struct(c, si, flags); write_struct(o, r.generic(), si, 0, 0, 0, false, flags); out_len = o.n; }
    r.nm = nm0;
    return;
  }
  // general path (noinline validator over a generic pointer)
  Cur c{r.generic(), start, r.end, 0, 0};
  SInfo si; read_struct(c, si, flags);
  if (c.err) { r.fail(c.err); return; }
  r.pos = c.pos; r.wat = 0xFFFFFFFFu;
  len = si.len; nc = si.nc;
  Out o{nullptr, 0};
  const bool hdr_nm = c.nm != 0;
  slow = si.renc || hdr_nm || true;  // general-path items are always written by write_struct
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

YDEV uint32_t wave_exscan(uint32_t v, uint32_t& total) {
  const uint32_t inc = wave_incl_scan_add(v);
  total = __shfl(inc, WAVE - 1, WAVE);
  return inc - v;
}

// parse pass over update i: counts (pass A) or record writes (pass B).  One
// non-inlined instance (LDS-typed pointer, results by value in registers).
struct UpdCount { uint32_t ns, nd; int err; uint32_t fb, nc; };
YDEV_NI UpdCount w_parse_update(LWave* L, int i, bool write, uint32_t sbase, uint32_t dbase, uint32_t flags) {
  WinRd r; r.init(L->in, L->ustart[i], (uint32_t)L->ustart[i] + L->ulen[i]);
  UpdCount uc{0, 0, 0, 0, 0};
  bool fb = false, nc = false;
  uint64_t prev_client = 0, prev_end = 0; bool have_prev = false;
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
        if (len == 0 || end > 0xFFFFFFFFull || len > 0xFFFFFFFFull) fb = true;
        if (have_prev && (client > prev_client || (client == prev_client && clock < prev_end))) fb = true;
        have_prev = true; prev_client = client; prev_end = end;
        if (snc) nc = true;
        if (write && !fb) {
          const uint32_t j = sbase + uc.ns;
          if (j < (uint32_t)W_S) {
            L->key[j] = ((uint64_t)(0xFFFFFFFFu - (uint32_t)client) << 32) | (uint32_t)clock;
            L->r_start[j] = (uint16_t)start; L->r_blen[j] = (uint16_t)(r.pos - start);
            L->r_len[j] = (uint32_t)len; L->r_ss[j] = (uint16_t)((i << 8) | (uc.ns & 0xFF));
            L->r_flag[j] = (uint8_t)(kind | (slow ? 4 : 0));
            L->r_out[j] = (uint16_t)olen;
          }
        }
        uc.ns++;
        if (uc.ns > 255) fb = true;  // seq is kept in 8 bits
      }
      clock = end;
    }
  }
  const uint64_t ncl = r.err ? 0 : r.vu();
  for (uint64_t q = 0; q < ncl && !r.err; q++) {
    const uint64_t cl = r.vu(), nr = r.vu();
    for (uint64_t k = 0; k < nr && !r.err; k++) {
      const uint64_t ck = r.vu(), ln = r.vu();
      if (r.err) break;
      if (cl > 0xFFFFFFFFull || ck + ln > 0xFFFFFFFFull) fb = true;
      if (write && !fb) {
        const uint32_t j = dbase + uc.nd;
        if (j < (uint32_t)W_D) { L->dkey[j] = ((uint64_t)(0xFFFFFFFFu - (uint32_t)cl) << 32) | (uint32_t)ck; L->dlen[j] = (uint32_t)ln; }
      }
      uc.nd++;
    }
  }
  uc.err = r.err; uc.fb = fb; uc.nc = nc;
  return uc;
}

}  // namespace ygm
