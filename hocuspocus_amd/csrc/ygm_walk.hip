// ygm_walk.hip -- encodeStateVectorFromUpdate / diffUpdate over a batch: the lane-per-document ring walker
// (ygm_doc_walk.hpp) and the state-vector table pre-pass; what the walker defers goes to the exact kernel k_doc
// (ygm_kernels.hip).  Its own file so the walker builds (and its experiment variants rebuild) alone.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ygm_docmeta.hpp"
#include "ygm_doc_walk.hpp"

#ifdef YGM_DIAG
// diagnostic build only (libygm_diag.so): walker census [0, 8) and per-section wave clocks [8, 13)
__device__ unsigned long long ygm_walk_diag[16];
#endif

namespace ygm {

// ======================================================================= SV / diff: lane-per-document ring walker
// ygm_doc_walk.hpp.  MODE 0 = encodeStateVectorFromUpdate (rule R-SV), 1 = diffUpdate (rule R-D).
// Wave w owns documents [n*w/G, n*(w+1)/G), cut into equal batches of <= DW_BATCH sorted largest first; a lane that
// finishes one takes the wave's next document at the following round start (offsets prefetched one round ahead,
// handed over by bpermute).  (Batches taken by ticket instead -- a shared counter, 64-256 documents each -- measured
// slower: profiles/r05_walk/README.md.)
// Outputs go to the document's slot (merge_slot): the header (a count known only at the end) is
// written right-aligned in front of the body at slot + 16.  Documents outside the walker's shape are
// appended to `defer_list` for k_doc.
// diffUpdate pre-pass: each document's state vector (decodeStateVector, Y@37797: a count, then
// (client, clock) varuints; a repeated client's last entry wins, as in its Map) parsed by one lane into
// a table sorted by client descending -- the order of the update's client blocks -- at tbl + 144 d as
// (client, clock) u32 pairs; tbl_n[d] = entries, or DW_TBL_BAD for a vector the walker leaves to the
// exact kernel (> DW_SVN entries, > DW_TBL_MAXB bytes, values >= 2^32, truncated, trailing bytes).
constexpr uint32_t DW_TBL_BAD = 0x80000000u;
constexpr uint32_t DW_TBL_MAXB = 160u;   // state-vector bytes staged per lane (16 entries of <= 10 bytes)
__global__ __launch_bounds__(WAVE) void k_sv_table(const uint8_t* __restrict__ sv_arena, const uint64_t* __restrict__ sv_off,
                                                  uint32_t n_docs, uint8_t* __restrict__ tbl, uint32_t* __restrict__ tbl_n) {
  __shared__ u32x4 buf[DW_TBL_MAXB / 16 + 1][WAVE];
  __shared__ uint32_t ec[DW_SVN][WAVE], ek[DW_SVN][WAVE];
  const uint32_t l = threadIdx.x, d = blockIdx.x * WAVE + l;
  if (d >= n_docs) return;
  const uint64_t sa = sv_off[d], sb = sv_off[d + 1];
  const uint32_t len = sb > sa ? (uint32_t)(sb - sa) : 0u;
  uint32_t bad = (sb < sa || len == 0u || len > DW_TBL_MAXB) ? 1u : 0u;
  const uint32_t o0 = (uint32_t)(sa & 15u);
  const u32x4* src = (const u32x4*)(sv_arena + (sa & ~15ull));
  const uint32_t np = bad ? 0u : (o0 + len + 15u) >> 4;
  for (uint32_t i = 0; i < np; i++) buf[i][l] = src[i];
  const uint8_t* b = (const uint8_t*)&buf[0][0];
  auto byte = [&](uint32_t i) -> uint32_t { return b[((i >> 4) * WAVE + l) * 16u + (i & 15u)]; };
  uint32_t pos = o0, end = o0 + (bad ? 0u : len);
  auto vu = [&]() -> uint32_t {   // varuint < 2^32 inside the vector, else bad
    uint64_t v = 0;
    for (uint32_t sh = 0;; sh += 7) {
      if (pos >= end || sh > 28) { bad = 1; return 0u; }
      const uint32_t x = byte(pos++);
      v |= (uint64_t)(x & 0x7Fu) << sh;
      if (x < 0x80u) break;
    }
    if (v >> 32) bad = 1;
    return (uint32_t)v;
  };
  const uint32_t cnt = bad ? 0u : vu();
  bad |= cnt > (uint32_t)DW_SVN ? 1u : 0u;
  uint32_t n = 0;
  for (uint32_t e = 0; e < (bad ? 0u : cnt); e++) {
    const uint32_t c = vu(), k = vu();
    if (bad) break;
    uint32_t j = 0;
    while (j < n && ec[j][l] > c) j++;
    if (j < n && ec[j][l] == c) { ek[j][l] = k; continue; }   // the last entry of a client wins
    for (uint32_t m = n; m > j; m--) { ec[m][l] = ec[m - 1][l]; ek[m][l] = ek[m - 1][l]; }
    ec[j][l] = c; ek[j][l] = k; n++;
  }
  bad |= pos != end ? 1u : 0u;   // trailing bytes: the exact kernel decides
  if (bad) { tbl_n[d] = DW_TBL_BAD; return; }
  uint64_t* t = (uint64_t*)(tbl + 144ull * d);
  for (uint32_t j = 0; j < n; j++) t[j] = ((uint64_t)ek[j][l] << 32) | ec[j][l];
  tbl_n[d] = n;
}

#ifndef YGM_DW_OUTEND
// diff output (pending header, copy run) written at the round's end, not at the next round's start: the commit at that
// start then sees the run's ring bytes released (written at the start, the run lagged a round behind the parse and
// the chunks staged past the ring were dropped and fetched again: diff 9.45 -> 7.49 GB fetched, 3.59 -> 3.29 ms)
#define YGM_DW_OUTEND 1
#endif
#ifndef YGM_DWX_NOST
#define YGM_DWX_NOST 0    // experiment only: copy runs without their stores (output wrong)
#endif
#ifndef YGM_DWX_NONEED
#define YGM_DWX_NONEED 0  // experiment only: chunk commits ignore the copy run's ring bytes (output wrong)
#endif
#ifndef YGM_DW_CB64
#define YGM_DW_CB64 1     // a document's chunks 64-byte aligned (each one half of a 128-byte line), not 16
#endif
#ifndef YGM_DW_PAIR
#define YGM_DW_PAIR 0     // 1: a round's staging ends on an even chunk (both halves of a line in one round); 2: rounds up
#endif
#ifndef YGM_DW_PAIR0
#define YGM_DW_PAIR0 2   // ... for the state vector (rounding down cost it 5 %: fewer chunks ahead)
#endif
#ifndef YGM_DW_PAIR1
#define YGM_DW_PAIR1 1   // ... for the diff
#endif
#ifndef YGM_DW_SVACC
#define YGM_DW_SVACC 1    // state vector: entries gathered in a 16-byte register chunk, stored aligned and whole
#endif
#ifndef YGM_DW_DACC
#define YGM_DW_DACC 0     // diff: every output byte through the 16-byte register chunk, stored aligned and whole
#endif
#ifndef YGM_DW_SPEC2
#define YGM_DW_SPEC2 0    // the next Item's info byte read beside this one's length byte (see the fast decoder)
#endif
#ifndef YGM_DWX_ALIGNST
#define YGM_DWX_ALIGNST 0 // experiment only: copy-run stores at 16-byte aligned positions (output wrong)
#endif
#ifndef YGM_DW_WPE0
#define YGM_DW_WPE0 2   // waves per SIMD the SV walker is compiled for (register budget 512 / waves)
#endif
#ifndef YGM_DW_WPE1
#define YGM_DW_WPE1 2   // ... the diff walker
#endif
template <int MODE>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(MODE == 0 ? YGM_DW_WPE0 : YGM_DW_WPE1))) void k_doc_walk(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off,
                                                  const uint8_t* __restrict__ tbl, const uint32_t* __restrict__ tbl_n,
                                                  uint32_t n_docs, uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                                                  uint64_t* __restrict__ out_len, int32_t* __restrict__ status, DocMeta* meta,
                                                  uint32_t* __restrict__ defer_list, uint64_t out_cap) {
  __shared__ DWLds L;
  uint32_t* ordk = L.ordk;
  const uint32_t l = threadIdx.x;
  const uint32_t D1 = (uint32_t)((uint64_t)n_docs * (blockIdx.x + 1) / gridDim.x);
  uint32_t bnext = (uint32_t)((uint64_t)n_docs * blockIdx.x / gridDim.x);   // wave-uniform: first document of the next batch
  uint32_t bbase = bnext, bn = 0, next = 0;                                  // the batch [bbase, bbase + bn); next: its first untaken entry

  // offsets of the next 64 documents of the batch (lane i: entry next + i), loaded one round ahead
  uint32_t pd = 0, ptn = 0;
  uint64_t pa = 0, pb = 0;
  auto prefetch = [&]() {
    pa = 0; pb = 0; ptn = 0; pd = 0;
    if (next + l < bn) {
      pd = bbase + (ordk[next + l] & 0xFFu);
      pa = doc_off[pd]; pb = doc_off[pd + 1];
      if (MODE == 1) ptn = tbl_n[pd];
    }
  };

  // ---- lane state
  uint32_t ph = WK_IDLE, d = 0, bad = 0;
  uint64_t da = 0, db = 0;                 // the document's bytes in `arena`
  // the lane's stream: MODE 1 first the document's state-vector table (chunks [0, tc): ring-relative bytes
  // [0, 8 nsv) = the table at tbl + 144 d), then the document; ring-relative byte r >= 64 tc is arena byte
  // cbase + r - 64 tc
  uint32_t tc = 0;
  uint64_t cbase = 0;                      // 16-byte aligned arena offset of the document's first chunk
  uint32_t srel = 0, q = 0, rb = 0;        // document start / parse position / document end, ring-relative
  uint32_t landed = 0, stg_n = 0, stg_k = 0, prev8 = 0;
  u32x4 g0 = {0u, 0u, 0u, 0u}, g1 = g0, g2 = g0, g3 = g0, g4 = g0, g5 = g0, g6 = g0, g7 = g0;   // staged chunks
  u32x4 g8 = g0, g9 = g0, g10 = g0, g11 = g0;
  u32x4 g12 = g0, g13 = g0, g14 = g0, g15 = g0;
  uint32_t n_left = 0, st_left = 0, client = 0, clock = 0, prevc = 0;
  bool have_prev = false;
  uint64_t slot = 0;                       // the document's output slot; t / tend / e_dst / cdst relative to it
  uint8_t* ob = out;                       // out + slot
  uint32_t tend = 0, t = 0;
  uint32_t count = 0;
  uint32_t sp = 0, str_end = 0, ph_after = 0;   // WK_STR: bytes [sp, str_end) of a long string still to check
  bool str_ascii = false;
  uint32_t clk = 0, cc = 0;                // MODE 0: the current block's state-vector clock
  bool stop = false, fst = false;          // fst: the document's first struct (its end counts even for a Skip)
  // pending output, written at the next round start.  MODE 0: entry (e_a, e_b); MODE 1: block header
  // (e_a, e_b, e_c) = (structs, client, clock) and, when e_pl > 0, the re-encoded prefix of a cut struct.
  bool e_on = false;
  uint32_t e_dst = 0;
  uint32_t e_a = 0, e_b = 0, e_c = 0, e_pl = 0, e_info = 0, e_oclk = 0, e_q = 0, e_ro_p = 0, e_ro_e = 0, e_clen = 0;
  // MODE 1: the state vector in registers: entries (sc[i], sk[i]), clients unique
  // copy run (ring bytes [cp, run_end) -> output at cdst)
  uint32_t nsv = 0, svc = 0;
  uint32_t sc[MODE == 1 ? DW_SVN : 1], sk[MODE == 1 ? DW_SVN : 1];
#pragma unroll
  for (int i = 0; i < (MODE == 1 ? DW_SVN : 1); i++) { sc[i] = 0; sk[i] = 0; }
  bool emitted = false, run_on = false;
  uint32_t cp = 0, run_end = 0, rs0 = 0;
  uint32_t cdst = 0, cd0 = 0;
  uint64_t payload = 0;
  uint32_t rounds = 0;
  // MODE 0 with YGM_DW_SVACC: output bytes [oq, oq + of) waiting in (oa0, oa1); oq 16-byte aligned, everything before it
  // stored.  Appends come in output order, so every 16-byte piece of the body is stored once, whole and aligned
  uint64_t oa0 = 0, oa1 = 0;
  uint32_t oq = 16, of = 0;
  auto put = [&](uint64_t lo, uint64_t hi, uint32_t n) {   // n <= 16 bytes, the bytes of (lo, hi) past n zero
    const uint32_t s = 8u * (of & 7u);
    const uint64_t x0 = lo << s, x1 = (hi << s) | ((lo >> (63u - s)) >> 1), x2 = (hi >> (63u - s)) >> 1;
    const bool hh = of >= 8u;
    oa0 |= hh ? 0ull : x0; oa1 |= hh ? x0 : x1;
    const uint64_t n0 = hh ? x1 : x2, n1 = hh ? x2 : 0ull;
    if (of + n >= 16u) { dw_st16(ob + oq, oa0, oa1); oq += 16u; oa0 = n0; oa1 = n1; }
    of = (of + n) & 15u;
  };
  (void)put;
#ifdef YGM_DIAG
  unsigned long long dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // lane-iterations: fast, general, not ready, idle, string; rounds, general iterations
#define WDG(i, v) dg[i] += (v)
  // wave shader-clock per section (wave-uniform code): commit, SV parse, grab + output + init, staging, parse
  unsigned long long tsec[5] = {0, 0, 0, 0, 0}, tprev = __builtin_amdgcn_s_memtime();
#define WSEC(i) do { const unsigned long long _n = __builtin_amdgcn_s_memtime(); tsec[i] += _n - tprev; tprev = _n; } while (0)
#else
#define WDG(i, v)
#define WSEC(i)
#endif

  // end of a client block (after its last struct): MODE 0 queues the block's state-vector entry,
  // MODE 1 closes the block's copy run
  auto block_end = [&]() {
    if (MODE == 0) {
      if (clk) {
        const uint32_t el = dw_vulen(cc) + dw_vulen(clk);
        if (t + el > tend) bad = 1;
        else { e_on = true; e_dst = t; e_a = cc; e_b = clk; t += el; count++; }
      }
      ph = --n_left ? WK_BLK : WK_FIN;
    } else {
      if (emitted) {   // the rest of the block, verbatim (Skips included)
        run_end = q;
        t = cd0 + (run_end - rs0);
        bad |= t > tend ? 1u : 0u;
      }
      ph = --n_left ? WK_BLK : WK_DS;
    }
  };
  // a block header: canonical blocks are strictly client-descending
  auto block_begin = [&](uint32_t nst, uint32_t cl, uint32_t ck) {
    bad |= (nst == 0u || (have_prev && cl >= prevc)) ? 1u : 0u;
    fst = !have_prev;
    prevc = cl; have_prev = true;
    st_left = nst; client = cl; clock = ck;
    if (MODE == 0) { cc = cl; stop = ck != 0u; clk = 0u; }
    else {   // the state-vector clock of the client: walk the descending table
      // (clients are unique in the table and its unused entries repeat entry 0, or hold clock 0: a
      // compare-select over all entries, no walk)
      uint32_t s = 0;
#pragma unroll
      for (int i = 0; i < (MODE == 1 ? DW_SVN : 1); i++) s = sc[i] == cl ? sk[i] : s;
      svc = s;
      emitted = false;
    }
    ph = WK_ST;
  };

  // the last round's pending header / cut prefix and the copy run (ring bytes [cp, q) -> output)
  auto flush_out = [&]() {
    if (e_on) {
      e_on = false;
      if (!bad) {
        uint64_t lo = dw_vu_enc(e_a), hi = 0;
        uint32_t at = dw_vulen(e_a);
        dw_app(lo, hi, at, e_b);
        if (MODE == 1) dw_app(lo, hi, at, e_c);
        if ((MODE == 0 && YGM_DW_SVACC) || (MODE == 1 && YGM_DW_DACC)) put(lo, hi, at);
        else dw_st16(ob + e_dst, lo, hi);
        if (MODE == 1 && YGM_DW_DACC && e_pl) {   // the re-encoded prefix of a cut struct, through the accumulator
          uint64_t plo = e_info, phi = 0;
          uint32_t pat = 1;
          if (e_info) { dw_app(plo, phi, pat, e_b); dw_app(plo, phi, pat, e_oclk); }
          put(plo, phi, pat);
          if (e_info && e_ro_e > e_ro_p) {   // the right origin, verbatim from the ring (<= 10 bytes)
            uint64_t rlo, rhi;
            dw_rd16(L, l, e_q + e_ro_p, rlo, rhi);
            const uint32_t n = e_ro_e - e_ro_p;
            rlo &= n >= 8u ? ~0ull : dw_lowmask(8u * n);
            rhi &= n > 8u ? dw_lowmask(8u * (n - 8u)) : 0ull;
            put(rlo, rhi, n);
          }
          put(dw_vu_enc(e_clen), 0ull, dw_vulen(e_clen));
        } else if (MODE == 1 && e_pl) {   // the re-encoded prefix of a cut struct
          uint64_t o = e_dst + at;
          ob[o++] = (uint8_t)e_info;
          if (e_info) {   // an item: origin (client, clock + off - 1), right origin verbatim
            o = dw_put_vu(ob, o, e_b);
            o = dw_put_vu(ob, o, e_oclk);
            for (uint32_t k = e_ro_p; k < e_ro_e; k++) ob[o++] = (uint8_t)dw_byte(L, l, e_q + k);
          }
          dw_put_vu(ob, o, e_clen);
        }
      }
    }
    if (MODE == 1 && YGM_DW_DACC && run_on) {   // the copy run through the accumulator: whole aligned output pieces only
      if (bad) run_on = false;
      else {
        const uint32_t done = ph == WK_STR ? sp : q;
        const bool fin = run_end <= done;
        uint32_t ce = fin ? run_end : done;
        if (!fin) {   // an open run: up to the last whole 16-byte output piece (the rest stays in the ring)
          const uint32_t tot = of + (ce - cp);
          ce = tot >= 16u ? cp + (tot & ~15u) - of : cp;
        }
        if (ce > cp) {
          if (cdst + (ce - cp) > tend) bad = 1;
          else {
            auto part = [&](uint32_t n) {   // n < 16 ring bytes at cp into the accumulator
              const u32x4 v = dw_ring16(L, l, cp);
              uint64_t vlo = ((uint64_t)v.y << 32) | v.x, vhi = ((uint64_t)v.w << 32) | v.z;
              vlo &= n >= 8u ? ~0ull : dw_lowmask(8u * n);
              vhi &= n > 8u ? dw_lowmask(8u * (n - 8u)) : 0ull;
              put(vlo, vhi, n);
              cp += n; cdst += n;
            };
            if (of) part(16u - of < ce - cp ? 16u - of : ce - cp);
            for (; cp + 16u <= ce; cp += 16u, cdst += 16u, oq += 16u) {   // (of == 0 here)
              const u32x4 v = (cp & 15u) ? dw_ring16(L, l, cp) : dw_piece(L, l, cp);
              __builtin_memcpy(ob + oq, &v, 16);
            }
            if (cp < ce) part(ce - cp);
          }
        }
        if (fin && !bad) run_on = false;
      }
    }
    if (MODE == 1 && !YGM_DW_DACC && run_on) {   // the copy run: ring bytes [cp, run_end) -> output at cdst
      if (bad) run_on = false;
      else {
        const uint32_t done = ph == WK_STR ? sp : q;
        const bool fin = run_end <= done;
        const uint32_t ce = fin ? run_end : (done & ~15u);   // an open run is written up to a ring piece boundary
        if (ce > cp) {
          if (cdst + (ce - cp) > tend) bad = 1;
          else {
            if (cp & 15u) {   // the head, up to the next ring piece boundary
              const u32x4 v = dw_ring16(L, l, cp);
              if (!YGM_DWX_NOST) __builtin_memcpy(ob + cdst, &v, 16);
              const uint32_t a = 16u - (cp & 15u) < ce - cp ? 16u - (cp & 15u) : ce - cp;
              cp += a; cdst += a;
            }
            for (; cp < ce; cp += 16u, cdst += 16u) {   // whole ring pieces
              const u32x4 v = dw_piece(L, l, cp);
              if (!YGM_DWX_NOST) __builtin_memcpy(ob + cdst, &v, 16);
            }
            cdst -= cp - ce; cp = ce;
          }
        }
        if (fin && !bad) run_on = false;
      }
    }
  };

  for (;;) {
    // ---- (0) a new batch of documents: sorted by size, largest first (the documents left at the end of a
    //      wave's range are its smallest: the last lanes to finish wait least)
    if (next >= bn && bnext < D1) {
      // equal batches of <= DW_BATCH: a short last batch would leave most lanes idle behind its largest document
      const uint32_t rem = D1 - bnext, nbat = (rem + DW_BATCH - 1u) / DW_BATCH;
      bbase = bnext; bn = (rem + nbat - 1u) / nbat; bnext = bbase + bn; next = 0;
      for (uint32_t e = l; e < (uint32_t)DW_BATCH; e += WAVE) {
        // key bytes + 1 (padding entries past bn: 0, sorted behind every document)
        const uint64_t sz = e < bn ? doc_off[bbase + e + 1] - doc_off[bbase + e] + 1ull : 0ull;
        ordk[e] = ((uint32_t)(sz < 0xFFFFFFull ? sz : 0xFFFFFFull) << 8) | e;
      }
      __syncthreads();
      for (uint32_t kk = 2; kk <= (uint32_t)DW_BATCH; kk <<= 1)
        for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
          for (uint32_t t2 = l; t2 < (uint32_t)DW_BATCH / 2; t2 += WAVE) {
            const uint32_t lo = ((t2 / jj) * 2 * jj) + (t2 % jj), hi = lo + jj;
            const uint32_t x = ordk[lo], y = ordk[hi];
            if ((x < y) == ((lo & kk) == 0)) { ordk[lo] = y; ordk[hi] = x; }   // descending
          }
          __syncthreads();
        }
      prefetch();
    }
    WSEC(4);
    // ---- (1) the chunks staged last round land in the ring (the compiler waits for their loads here)
    //      -- those whose ring slot is free by now: staging runs DW_AHEAD chunks past the ring, betting on this
    //      round's consumption; a chunk that lost the bet is dropped here and staged again
    if (stg_n) {
      uint32_t need = ph == WK_STR ? sp : (MODE == 1 && ph == WK_SVN) ? 0u : q;   // (the table stays until copied)
      if (!YGM_DWX_NONEED && run_on && cp < need) need = cp;
      if (!YGM_DWX_NONEED && MODE == 1 && e_on && e_q < need) need = e_q;   // the pending cut struct's right origin is copied from the ring
      const uint32_t lim = (need >> 6) + DW_S;
      if (stg_k + stg_n > lim) stg_n = lim > stg_k ? lim - stg_k : 0u;
    }
    if (stg_n) {
      // the document part [vlo, vhi) of chunk k is checked (table chunks: none)
      auto vlo = [&](uint32_t k) { return srel > 64u * k ? (srel - 64u * k < 64u ? srel - 64u * k : 64u) : 0u; };
      auto vhi = [&](uint32_t k) { return k < tc ? 0u : (rb - 64u * k < 64u ? rb - 64u * k : 64u); };
      dw_commit<MODE == 1>(L, l, stg_k, g0, g1, g2, g3, vlo(stg_k), vhi(stg_k), prev8, bad);
      if (stg_n > 1u) {
        const uint32_t k1 = stg_k + 1u;
        dw_commit<MODE == 1>(L, l, k1, g4, g5, g6, g7, vlo(k1), vhi(k1), prev8, bad);
      }
      if (stg_n > 2u) {
        const uint32_t k2 = stg_k + 2u;
        dw_commit<MODE == 1>(L, l, k2, g8, g9, g10, g11, vlo(k2), vhi(k2), prev8, bad);
      }
      if (DW_STG > 3u && stg_n > 3u) {
        const uint32_t k3 = stg_k + 3u;
        dw_commit<MODE == 1>(L, l, k3, g12, g13, g14, g15, vlo(k3), vhi(k3), prev8, bad);
      }
      landed = stg_k + stg_n;
      stg_n = 0;
    }
    WSEC(0);
    // ---- (1b) diff: a landed state-vector table moves from the ring to the lane's table, the document follows
    if (MODE == 1) {
      const bool cpy = ph == WK_SVN && landed >= tc;
      const uint64_t cm = __ballot(cpy);
      if (cm && cpy) {
#pragma unroll
        for (int i = 0; i < (MODE == 1 ? DW_SVN : 1); i++) {   // unused entries: copies of entry 0 (or clock 0)
          const uint64_t w = (uint32_t)i < nsv ? dw_word(L, l, 8u * (uint32_t)i) : (i ? ((uint64_t)sk[0] << 32 | sc[0]) : 0ull);
          sc[i] = (uint32_t)w; sk[i] = (uint32_t)(w >> 32);
        }
        ph = WK_UPD;
      }
    }
    WSEC(1);
    // ---- (2) lanes that are idle or finishing take the wave's next documents
    const bool want = ph == WK_IDLE || ph == WK_FIN;
    const uint64_t wm = __ballot(want);
    const uint32_t rank = lanes_below(wm) & 63u;
    const uint64_t na = dw_shfl64(pa, rank), nb = dw_shfl64(pb, rank);
    const uint32_t nd = (uint32_t)__shfl((int)pd, (int)rank);
    const uint32_t ntn = MODE == 1 ? (uint32_t)__shfl((int)ptn, (int)rank) : 0u;
    const uint32_t avail = bn - next;
    const bool got = want && rank < avail;
    const uint32_t npop = (uint32_t)__popcll(wm);
    next += npop < avail ? npop : avail;
    // ---- (3) output of the last round: pending header / entry, the copy run, finished documents
    // Output stores are 16 bytes wide, whatever the byte count: the bytes past a store's valid part are
    // overwritten by the document's next store (a lane writes its output in increasing order) or lie
    // in the slot's last 16 bytes, which tend keeps free
    if (!YGM_DW_OUTEND) flush_out();
    if (ph == WK_FIN) {
      const uint64_t bm = __ballot(bad != 0u);   // (only finishing lanes reach here)
      if (bm) {
        uint32_t base = 0;
        if (l == (uint32_t)__builtin_ctzll(bm)) base = atomicAdd(&meta->lean_defer, (uint32_t)__popcll(bm));
        base = (uint32_t)__shfl((int)base, (int)__builtin_ctzll(bm));
        if (bad) { defer_list[base + lanes_below(bm)] = d; status[d] = ST_FALLBACK; }
      }
      if (((MODE == 0 && YGM_DW_SVACC) || (MODE == 1 && YGM_DW_DACC)) && !bad && of) dw_st16(ob + oq, oa0, oa1);   // the body's last piece
      if (!bad) {   // the count, right-aligned in the slot's first 16 bytes (an aligned store)
        const uint32_t hl = dw_vulen(count);
        const uint64_t c = dw_vu_enc(count);
        dw_st16(ob, 0ull, c << (64u - 8u * hl));
        out_off[d] = slot + 16u - hl; out_len[d] = hl + (t - 16u); status[d] = ST_OK;
        payload += hl + (t - 16u);
      }
      ph = WK_IDLE; run_on = false; e_on = false;
    }
    // ---- (4) new documents
    if (got) {
      d = nd; bad = 0; da = na; db = nb; count = 0; emitted = false; have_prev = false; nsv = 0;
      oa0 = 0; oa1 = 0; oq = 16u; of = 0;
      slot = merge_slot(da, d);
      ob = out + slot;
      const uint64_t cap = merge_slot_cap(db - da), room = out_cap > slot ? out_cap - slot : 0ull;
      const uint64_t lim = cap < room ? cap : room;
      tend = lim > 16u ? (uint32_t)(lim - 16u) : 0u;   // (16 bytes of slack for the wide stores)
      t = 16u;   // the header (a count known only at the end) goes right-aligned in front of the body
      nsv = MODE == 1 && ntn <= (uint32_t)DW_SVN ? ntn : 0u;
      bad |= (MODE == 1 && ntn > (uint32_t)DW_SVN) ? 1u : 0u;   // (DW_TBL_BAD: the exact kernel)
      tc = (8u * nsv + 63u) >> 6;
      if (MODE == 1 && !tc) {   // an empty state vector: every client at clock 0
#pragma unroll
        for (int i = 0; i < (MODE == 1 ? DW_SVN : 1); i++) sk[i] = 0u;
      }
      cbase = da & (YGM_DW_CB64 ? ~63ull : ~15ull);
      srel = 64u * tc + (uint32_t)(da - cbase); q = srel; rb = 64u * tc + (uint32_t)(db - cbase);
      landed = 0; stg_n = 0; prev8 = 0;
      bad |= (db < da || ((db - da) >> 30)) ? 1u : 0u;
      ph = tc ? WK_SVN : WK_UPD;
    }
    if (__ballot(ph != WK_IDLE) == 0 && next >= bn && bnext >= D1) break;
    WSEC(2);
    // ---- (5) stage the next chunks of the segment (up to three; the ring keeps DW_S)
    if (ph != WK_IDLE && ph != WK_FIN) {
      uint32_t need = ph == WK_STR ? sp : (MODE == 1 && ph == WK_SVN) ? 0u : q;
      if (run_on && cp < need) need = cp;
      const uint32_t nch = (rb + 63u) >> 6;
      const uint32_t wk = (need >> 6) + DW_S + DW_AHEAD < nch ? (need >> 6) + DW_S + DW_AHEAD : nch;
      uint32_t n = wk > landed ? (wk - landed < DW_STG ? wk - landed : DW_STG) : 0u;
      // (with CB64 the document's chunk j is the half (cbase / 64 + j) & 1 of its 128-byte line; chunk k = tc + j)
      const uint32_t lpar = ((uint32_t)(cbase >> 6) - tc) & 1u;
      constexpr int PAIR = MODE == 0 ? YGM_DW_PAIR0 : YGM_DW_PAIR1;
      if (PAIR == 1 && n > 1u && ((landed + n + lpar) & 1u)) n--;
      if (PAIR == 2 && n && n < DW_STG && ((landed + n + lpar) & 1u) && landed + n < nch) n++;
      stg_k = landed; stg_n = n;
      auto chunk = [&](uint32_t k) -> const u32x4* {
        return (const u32x4*)(MODE == 1 && k < tc ? tbl + 144ull * d + 64u * k : arena + cbase + 64ull * (k - tc));
      };
      if (n >= 1u) { const u32x4* p = chunk(landed); g0 = p[0]; g1 = p[1]; g2 = p[2]; g3 = p[3]; }
      if (n >= 2u) { const u32x4* p = chunk(landed + 1u); g4 = p[0]; g5 = p[1]; g6 = p[2]; g7 = p[3]; }
      if (n >= 3u) { const u32x4* p = chunk(landed + 2u); g8 = p[0]; g9 = p[1]; g10 = p[2]; g11 = p[3]; }
      if (DW_STG > 3u && n >= 4u) { const u32x4* p = chunk(landed + 3u); g12 = p[0]; g13 = p[1]; g14 = p[2]; g15 = p[3]; }
    }
    // ---- (6) offsets of the documents the next round hands out
    prefetch();
    WSEC(3);
    // ---- (7) parse: per lane and iteration one unit, by the fast decoder when it has the common shape
    //      (an Item with origin(s) and a one-byte String / Deleted length inside 32 bytes, a block header
    //      of a <= 2-byte count and a one-byte clock, a one-byte update header, an empty delete set),
    //      else by the general decoder -- which then runs for the lanes that need it only
#pragma unroll 1
    for (int it = 0; it < (MODE == 1 ? DW_R - 1 : DW_R); it++) {   // (diff: shorter rounds, its output waits for them)
      if (bad && ph != WK_IDLE) ph = WK_FIN;
      // block headers are decoded on even iterations only: the wave skips the header decoder every other
      // iteration (with 64 lanes some lane is at a header in most iterations; a lane waits one at most)
      const bool blk_it = (it & 1) == 0;
#ifdef YGM_DIAG
      const uint32_t ph0 = ph;
#endif
      const uint32_t lend = landed << 6;
      const bool rdy = (q + 64u <= lend) || (lend >= rb);   // the general decoder reads up to 64 bytes ahead
      // the fast decoders take a unit whose bytes have all landed (masks past lend are stale: a unit
      // that ends there is refused and retried)
      const uint32_t avl = lend > q ? lend - q : 0u;
      bool done = false;
      if (avl && (ph == WK_ST || ph == WK_BLK || ph == WK_UPD || (MODE == 1 && ph == WK_DS))) {
        const uint32_t sq = q & 63u;
        uint64_t m0, m1;
        dw_mask2r(L, l, q, m0, m1);
        // bytes q .. q + 63 (chunks past the segment may hold stale masks: every unit is checked against rb)
        const uint64_t w64 = (m0 >> sq) | ((m1 << (63u - sq)) << 1);
        const uint32_t w32 = (uint32_t)w64;
        const uint32_t b0 = dw_byte(L, l, q);
        if (ph == WK_ST) {   // Items with origin(s), one-byte String (ASCII) / Deleted length, inside 32 bytes:
                             // up to DW_U from the same 64-byte window.  Block ends and (diff) block headers are
                             // handled once after the loop, not in each of its unrolled steps
          uint32_t qo = 0, bb = b0;
          const uint32_t lim = avl < 64u ? avl : 64u;   // a unit ends inside the landed bytes and the 64-byte window
          bool go = true;   // (ph == WK_ST implies st_left >= 1)
          bool pe = false;  // diff: the step that stopped the loop is the block's first struct past the state vector
          uint32_t pe_end = 0, pe_ce = 0;
          // YGM_DW_SPEC2: the bytes one and two past an Item's length byte are read beside it -- the next Item's info byte
          // when this one is Deleted content / a one-character string -- so the chain holds one dependent LDS read
          // per Item, not two
          uint32_t nbs = 0;
          bool spec = false;
#pragma unroll
          for (int u = 0; u < (MODE == 1 ? DW_U1 : DW_U); u++) {
            const uint32_t wq = (uint32_t)(w64 >> qo);
            const uint32_t tt = wq >> 1, x2 = tt & (tt - 1u), x3 = x2 & (x2 - 1u), x4 = x3 & (x3 - 1u);
            if (u >= 1) {
              if (YGM_DW_SPEC2 && spec) bb = nbs;
              else bb = dw_byte(L, l, q);
            }
            const uint32_t hoh = bb >> 6, ref = bb & 0x3Fu;
            const uint32_t cpos = (uint32_t)__builtin_ctz((hoh == 3u ? x4 : x2) | 0x80000000u) + 2u;   // after the origins
            const uint32_t cq = cpos & 31u;
            const uint32_t lv = dw_byte(L, l, q + cq);
            uint32_t nb1 = 0, nb2 = 0;
            if (YGM_DW_SPEC2) { nb1 = dw_byte(L, l, q + cq + 1u); nb2 = dw_byte(L, l, q + cq + 2u); }
            const bool isS = ref == 4u;
            const uint32_t end = cq + 1u + (isS ? lv : 0u);
            // the string's bytes are ASCII: every one of them ends a varuint (no clear bit among the lv after the length)
            // (bits past the 32-bit window never count: end <= 32 below keeps the string inside it)
            const bool asc = (uint32_t)__builtin_ctz((~wq >> ((cq + 1u) & 31u)) | 0x80000000u) >= lv;
            const uint32_t ce = clock + lv;
            // (boolean terms as comparisons: lane masks combined by the scalar unit, no VALU materialisation)
            bool ok = go & (hoh != 0u) & (isS | (ref == 1u)) & (cpos < 31u) & (__builtin_amdgcn_ubfe(wq, cq, 1) != 0u) &
                      (lv != 0u) & (end <= 32u) & (!isS | asc) & (ce >= clock) & (qo + end <= lim);
            if (MODE == 0) ok &= (st_left != 1u) | !e_on;   // the block's last struct queues its entry
            else {
              const bool emit = !emitted & (ce > svc);
              // a cut struct (svc > clock) or a header / copy run still in flight: the general decoder / a later round
              if (ok & emit) { pe = (svc <= clock) & !e_on & !run_on; pe_end = end; pe_ce = ce; }
              ok &= !emit;
            }
            if (ok) {
              WDG(7, 1);   // Items taken by the fast decoder
              if (MODE == 0) {
                clk = stop ? clk : ce;   // (no Skips here: the first-struct seeding is the same)
                fst = false;
              }
              clock = ce;
              q += end; qo += end;
              --st_left;
            }
            go = ok && st_left != 0u;
            if (YGM_DW_SPEC2) { spec = !isS | (lv == 1u); nbs = isS ? nb2 : nb1; }
          }
          if (MODE == 1 && pe) {   // the first struct of the block past the state vector (rule R-D): the block
                                   // header, then the rest of the block as a copy run from this struct on
            const uint32_t hl = dw_vulen(st_left) + dw_vulen(client) + dw_vulen(clock);
            if (t + hl > tend) bad = 1;
            else {
              e_on = true; e_dst = t; e_a = st_left; e_b = client; e_c = clock; e_pl = 0; e_q = q;
              t += hl;
              run_on = true; cp = q; rs0 = q; cdst = t; cd0 = t; run_end = DW_OPEN;
              emitted = true; count++;
            }
            clock = pe_ce;
            q += pe_end;
            --st_left;
          }
          done = qo != 0u || pe;
          if (st_left == 0u) block_end();
        } else if (ph == WK_BLK && blk_it) {   // block header: <= 2-byte count, <= 5-byte client, one-byte clock
          const uint32_t y = w32 & (w32 - 1u), z = y & (y - 1u);
          const uint32_t e1 = (uint32_t)__builtin_ctz(w32 | 0x80000000u), e2 = (uint32_t)__builtin_ctz(y | 0x80000000u);
          const uint32_t e3 = (uint32_t)__builtin_ctz(z | 0x80000000u);
          const uint32_t b1 = dw_byte(L, l, q + 1u);
          const uint32_t cn = e2 - e1;   // client bytes
          const uint64_t cw = dw_rd8(L, l, q + (e1 & 1u) + 1u);
          const uint32_t nst = e1 == 0u ? b0 : ((b0 & 0x7Fu) | (b1 << 7));
          const uint32_t ok = (z != 0u) & (e1 <= 1u) & (e3 == e2 + 1u) & (cn - 1u <= 4u) & !((cn == 5u) & (((uint32_t)(cw >> 32) & 0x70u) != 0u)) &
                              (e3 < avl);
          if (ok) {
            done = true;
            const uint32_t cl = (uint32_t)pext7(cw, cn);
            const uint32_t ck = (uint32_t)(cw >> (8u * (cn & 7u))) & 0x7Fu;
            q += e3 + 1u;
            block_begin(nst, cl, ck);
          }
        } else if (ph == WK_UPD) {
          if (w32 & 1u) {
            done = true;
            q += 1u;
            if (b0) { n_left = b0; have_prev = false; ph = WK_BLK; }
            else ph = MODE == 1 ? WK_DS : WK_FIN;
          }
        } else if (MODE == 1 && ph == WK_DS && (w32 & 1u) && b0 == 0u && !run_on) {   // the empty delete set ("00") (avl >= 1)
          done = true;
          run_on = true; cp = q; rs0 = q; cdst = t; cd0 = t;
          q += 1u; run_end = q; t += 1u;
          bad |= t > tend ? 1u : 0u;
          ph = WK_FIN;
        }
        if (q > rb) bad = 1;
      }
#ifdef YGM_DIAG
      {   // one class per lane-iteration, from the phase it started in
        const bool idl = ph0 == WK_IDLE || ph0 == WK_FIN || ph0 == WK_SVN;
        WDG(0, done ? 1 : 0);
        WDG(3, (!done && idl) ? 1 : 0);
        WDG(4, (!done && !idl && ph0 == WK_STR) ? 1 : 0);
        WDG(2, (!done && !idl && ph0 != WK_STR && !rdy) ? 1 : 0);
        WDG(1, (!done && !idl && ph0 != WK_STR && rdy) ? 1 : 0);
      }
#endif
#ifdef YGM_DIAG
      if (l == 0) dg[6] += __ballot(!done && rdy && ph != WK_IDLE && ph != WK_FIN && ph != WK_SVN && ph != WK_STR) ? 1 : 0;
#endif
      if (!done && ph == WK_STR) {   // the rest of a long string (or binary): checked against the chunk masks
        if (sp < lend) {
          const uint64_t wn = dw_win(L, l, sp, landed);
          uint32_t n = str_end - sp;
          if (n > lend - sp) n = lend - sp;
          if (n > 64u) n = 64u;
          if (str_ascii && ((~wn) & dw_lowmask(n))) bad = 1;
          sp += n;
          if (sp == str_end) ph = ph_after;
        }
      } else if (!done && rdy && ph != WK_IDLE && ph != WK_FIN && ph != WK_SVN && (blk_it || ph != WK_BLK)) {   // ---- the general decoder
        const uint64_t win = dw_win(L, l, q, landed);
        uint64_t lo, hi;
        dw_rd16(L, l, q, lo, hi);
        if (ph == WK_ST) {
          const uint32_t info = (uint32_t)lo & 0xFFu;
          const uint64_t w1 = win & ~1ull;   // terminators after the info byte
          uint32_t len = 0, end = 0, kind = K_ITEM, ro_p = 0, ro_e = 0, cdata = 0, ref = 0, ho = 0, hr = 0;
          bool spill = false, sasc = true;
          if ((info & 31u) == 0u || info == 10u) {   // GC / Skip: varuint length
            kind = info == 10u ? K_SKIP : K_GC;
            bad |= (info != 0u && info != 10u) ? 1u : 0u;   // GC written back as info 0 by yjs
            const uint32_t e = dw_ctz(w1);
            len = dw_val(dw_at(lo, hi, 1u), e, bad);
            bad |= len == 0u ? 1u : 0u;
            end = e + 1u;
          } else {
            ref = info & 31u; ho = (info >> 7) & 1u; hr = (info >> 6) & 1u;
            bad |= ((info & 0xC0u) && (info & 0x20u)) ? 1u : 0u;   // yjs drops the bit on re-encode
            uint32_t cs;
            if (ho | hr) {   // origin and/or right origin: two varuints each
              uint64_t x = w1;
              const uint32_t t2 = dw_ctz(x & (x - 1ull));
              x &= x - 1ull; x &= x - 1ull; x &= x - 1ull;
              const uint32_t t4 = dw_ctz(x);
              cs = ((ho & hr) ? t4 : t2) + 1u;
              ro_p = ho ? t2 + 1u : 1u; ro_e = cs;
            } else {   // parent: parentInfo 1 -> y-key string, 0 -> parent id; parentSub string when bit 0x20
              const uint32_t pe = dw_ctz(w1);
              const uint32_t pi = dw_val(dw_at(lo, hi, 1u), pe, bad);
              bad |= pi > 1u ? 1u : 0u;
              uint32_t p = pe + 1u;
              if (pi == 1u) p = dw_str(L, l, q, win, lo, hi, p < 63u ? p : 63u, bad);
              else { uint64_t x = dw_from(win, p); x &= x - 1ull; p = dw_ctz(x) + 1u; }
              if (info & 0x20u) p = dw_str(L, l, q, win, lo, hi, p < 63u ? p : 63u, bad);
              cs = p;
            }
            bad |= cs >= 60u ? 1u : 0u;
            const uint32_t csx = cs < 56u ? cs : 56u;
            const uint32_t ce = dw_ctz(dw_from(win, csx));
            const uint32_t v = dw_val(dw_bytes_at(L, l, q, lo, hi, csx), ce - csx + 1u, bad);
            const uint32_t cend = ce + 1u;
            if (ref == 1u) {   // ContentDeleted
              len = v; end = cend;
              bad |= v == 0u ? 1u : 0u;
            } else if (ref == 4u || ref == 3u) {   // ContentString (ASCII: UTF-16 length = bytes) / ContentBinary
              sasc = ref == 4u;
              len = sasc ? v : 1u; cdata = cend; end = cend + v;
              bad |= (sasc && v == 0u) ? 1u : 0u;
              if (end <= 64u) { if (sasc && cdata < 64u && ((~win >> cdata) & dw_lowmask(v))) bad = 1; }
              else { spill = true; if (sasc && cdata < 64u && (~win >> cdata)) bad = 1; }
            } else if (ref == 7u) {   // ContentType: typeRef, key for XmlElement / XmlHook
              len = 1u; end = cend;
              bad |= v > 6u ? 1u : 0u;
              if (v == 3u || v == 5u) end = dw_str(L, l, q, win, lo, hi, cend < 63u ? cend : 63u, bad);
            } else bad = 1;   // JSON / Embed / Format / Any / Doc: the exact kernel
          }
          if (!bad) {
            const uint64_t ce64 = (uint64_t)clock + len;
            bad |= (ce64 >> 32) ? 1u : 0u;
            bool emit = false, stall;
            if (MODE == 0) stall = st_left == 1u && e_on;   // this block's entry needs the entry slot
            else {
              emit = !emitted && kind != K_SKIP && ce64 > svc;
              stall = emit && (e_on || run_on);   // one block header / copy run in flight per lane
            }
            if (!stall && !bad) {
              const uint32_t q0 = q;
              if (MODE == 0) {
                if (fst && !stop) clk = (uint32_t)ce64;   // yjs seeds the count with the first struct, Skip or not
                fst = false;
                if (kind == K_SKIP) stop = true;
                if (!stop) clk = (uint32_t)ce64;
              } else if (emit) {   // the first struct of the client past the state vector (rule R-D)
                const uint32_t off = svc > clock ? svc - clock : 0u;
                const uint32_t hck = clock + off;
                const uint32_t hl = dw_vulen(st_left) + dw_vulen(client) + dw_vulen(hck);
                uint32_t pl = 0, rstart = q;
                if (off) {   // cut: GC -> GC(len - off); Deleted / String -> origin (client, clock + off - 1)
                  if (kind == K_GC) { e_info = 0; e_clen = len - off; pl = 1u + dw_vulen(e_clen); rstart = q + end; }
                  else {
                    e_info = ref | 0x80u | (hr ? 0x40u : 0u) | ((!ho && !hr && (info & 0x20u)) ? 0x20u : 0u);
                    e_oclk = clock + off - 1u;
                    e_ro_p = hr ? ro_p : 0u; e_ro_e = hr ? ro_e : 0u;
                    e_clen = len - off;
                    pl = 1u + dw_vulen(client) + dw_vulen(e_oclk) + (e_ro_e - e_ro_p) + dw_vulen(e_clen);
                    rstart = ref == 4u ? q + cdata + off : q + end;
                  }
                }
                if (t + hl + pl > tend) bad = 1;
                else {
                  e_on = true; e_dst = t; e_a = st_left; e_b = client; e_c = hck; e_pl = pl; e_q = q;
                  t += hl + pl;
                  run_on = true; cp = rstart; rs0 = rstart; cdst = t; cd0 = t; run_end = DW_OPEN;
                  emitted = true; count++;
                }
              }
              clock = (uint32_t)ce64;
              q += end;
              if (--st_left == 0u) block_end();
              if (spill) { sp = q0 + 64u; str_end = q0 + end; str_ascii = sasc; ph_after = ph; ph = WK_STR; }
            }
          }
        } else {   // headers and delete-set entries: up to three varuints
          uint64_t x = win;
          const uint32_t e1 = dw_ctz(x); x &= x - 1ull;
          const uint32_t e2 = dw_ctz(x); x &= x - 1ull;
          const uint32_t e3 = dw_ctz(x);
          uint32_t b1 = 0, b2 = e2 >= 16u ? 1u : 0u, b3 = e3 >= 16u ? 1u : 0u;
          const uint32_t v1 = dw_val(lo, e1 + 1u, b1);
          const uint32_t v2 = dw_val(dw_at(lo, hi, e1 + 1u < 15u ? e1 + 1u : 15u), e2 - e1, b2);
          const uint32_t v3 = dw_val(dw_at(lo, hi, e2 + 1u < 15u ? e2 + 1u : 15u), e3 - e2, b3);
          if (ph == WK_UPD) {
            bad |= b1;
            q += e1 + 1u;
            if (v1) { n_left = v1; have_prev = false; ph = WK_BLK; }
            else ph = MODE == 1 ? WK_DS : WK_FIN;
          } else if (ph == WK_DS) {   // the delete set is copied verbatim (readDeleteSet + writeDeleteSet)
            if (!run_on) {
              bad |= b1;
              const uint32_t q0 = q;
              q += e1 + 1u;
              run_on = true; cp = q0; rs0 = q0; cdst = t; cd0 = t; run_end = DW_OPEN;
              if (v1) { n_left = v1; have_prev = false; ph = WK_DSC; }
              else { run_end = q; t = cd0 + (q - q0); bad |= t > tend ? 1u : 0u; ph = WK_FIN; }
            }
          } else if (ph == WK_BLK) {   // client block header: structs, client, first clock
            bad |= b1 | b2 | b3;
            q += e3 + 1u;
            if (!bad) block_begin(v1, v2, v3);
          } else if (ph == WK_DSC) {   // delete-set client: >= 1 range, clients strictly descending
            bad |= b1 | b2;
            q += e2 + 1u;
            bad |= (v2 == 0u || (have_prev && v1 >= prevc)) ? 1u : 0u;
            prevc = v1; have_prev = true;
            st_left = v2; ph = WK_DSR;
          } else {   // WK_DSR: one (clock, len) range, copied verbatim
            bad |= e2 >= 64u ? 1u : 0u;
            q += e2 + 1u;
            if (--st_left == 0u) {
              if (--n_left == 0u) { run_end = q; t = cd0 + (q - rs0); bad |= t > tend ? 1u : 0u; ph = WK_FIN; }
              else ph = WK_DSC;
            }
          }
        }
        if (q > rb) bad = 1;
      }
    }
    if (YGM_DW_OUTEND) flush_out();   // (at the round's end: the next commit sees the run's ring bytes released)
    if (++rounds > (1u << 26)) { if (l == 0) atomicOr(&meta->fault, 1u); break; }
  }
  payload = wave_sum(payload);
  if (l == 0 && payload) add_payload(meta, blockIdx.x, payload);
#ifdef YGM_DIAG
  dg[5] = l == 0 ? rounds : 0;
  for (int i = 0; i < 8; i++) { const unsigned long long v = wave_sum(dg[i]); if (l == 0) atomicAdd(&ygm_walk_diag[i], v); }
  if (l == 0) for (int i = 0; i < 5; i++) atomicAdd(&ygm_walk_diag[8 + i], tsec[i]);
#endif
#undef WDG
}

}  // namespace ygm

extern "C" {

using namespace ygm;

#ifdef YGM_DIAG
int ygm_walk_diag_read(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ygm_walk_diag), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(ygm_walk_diag), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

size_t ygm_k_sv_table_bytes(uint32_t n_docs) { return 144ull * n_docs + 64; }
int ygm_k_launch_doc_lean(int mode, const uint8_t* arena, uint64_t arena_bytes, const uint64_t* doc_off, const uint8_t* sv_arena,
                          uint64_t sv_bytes, const uint64_t* sv_off, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                          uint64_t* out_len, int32_t* status, void* meta, uint32_t* defer_list, uint64_t out_cap, uint8_t* tbl,
                          uint32_t* tbl_n, hipStream_t s) {
  (void)arena_bytes; (void)sv_bytes; (void)flags;   // segments are read in 64-byte chunks: 64 bytes of tail padding (ygm.h)
  if (n_docs == 0) return 0;
  const int n_cu = (int)device_cus();
  const char* env = getenv("YGM_WALK_WAVES_PER_CU");
  // resident waves per CU: 4 SIMDs x the waves per SIMD the walker is compiled for (its LDS fits them)
  const uint32_t wpc = env ? (uint32_t)atoi(env) : 4u * (mode == 0 ? YGM_DW_WPE0 : YGM_DW_WPE1);
  const uint32_t waves = (n_docs + WAVE - 1) / WAVE, cap = (uint32_t)n_cu * (wpc ? wpc : 1u);
  uint32_t grid = waves < cap ? waves : cap;
  const char* genv = getenv("YGM_WALK_GRID");   // testing: a small grid gives every lane many documents
  if (genv && atoi(genv) > 0 && (uint32_t)atoi(genv) < grid) grid = (uint32_t)atoi(genv);
  if (mode == 0)
    hipLaunchKernelGGL(k_doc_walk<0>, dim3(grid), dim3(WAVE), 0, s, arena, doc_off, (const uint8_t*)nullptr, (const uint32_t*)nullptr,
                       n_docs, out, out_off, out_len, status, (DocMeta*)meta, defer_list, out_cap);
  else {
    hipLaunchKernelGGL(k_sv_table, dim3(waves), dim3(WAVE), 0, s, sv_arena, sv_off, n_docs, tbl, tbl_n);
    hipLaunchKernelGGL(k_doc_walk<1>, dim3(grid), dim3(WAVE), 0, s, arena, doc_off, (const uint8_t*)tbl, (const uint32_t*)tbl_n, n_docs,
                       out, out_off, out_len, status, (DocMeta*)meta, defer_list, out_cap);
  }
  return launch_rc(__func__);
}

}  // extern "C"
