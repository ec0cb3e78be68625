// ygm_kernels.hip -- gfx950 kernels of the batched Yjs update engine.
//
//  k_doc         encodeStateVectorFromUpdate / diffUpdate, one lane per document (yjs Y@37728 / Y@40711):
//                the exact kernel for what the ring walker (ygm_walk.hip) defers
//  k_merge_fast  mergeUpdates, one workgroup per document, all state in LDS:
//                stage -> parse (lane per update) -> bitonic sort of struct
//                keys (client desc, clock asc) -> provenance scan (Skip gaps,
//                GC coalescing, rule R-M of SURVEY.md App. B.5) -> delete-set
//                segmented max-scan union (rule R-DS) -> emit
//  k_merge_seq   mergeUpdates, exact sequential replay (one lane per document)
//                for documents the fast path cannot prove overlap-free
//
// Output placement: every kernel writes a packed arena in document order using
// decoupled look-back over tiles taken in ticket order (ygm_common.hpp), so a
// batch is ONE pass over the input; the sequential kernel appends after the
// fast region through an atomic cursor (offsets are reported per document).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>

#include "ygm_common.hpp"
#include "ygm_merge_seq.hpp"
#include "ygm_merge_wave.hpp"
#include "ygm_merge_lean.hpp"
#include "ygm_docmeta.hpp"
#include "ygm_doc_walk.hpp"   // (its byte-window helpers: dw_at, dw_fsh, ...)
#include "ygm_merge_big.hpp"
#include "ygm_seqdoc.hpp"
#include "ygm_v1.hpp"

#ifdef YGM_DIAG
// diagnostic build only (libygm_diag.so): per-phase shader-clock sums of k_merge_fast
__device__ unsigned long long ygm_diag[32];
#define DIAG_T0 unsigned long long _dt = __builtin_amdgcn_s_memtime();
#define DIAG(i) do { if (threadIdx.x == 0) { unsigned long long _n = __builtin_amdgcn_s_memtime(); atomicAdd(&ygm_diag[i], _n - _dt); _dt = _n; } } while (0)
#define DIAGW(i) do { if ((threadIdx.x & 63) == 0) { unsigned long long _n = __builtin_amdgcn_s_memtime(); atomicAdd(&ygm_diag[8 + (i)], _n - _dt); _dt = _n; } } while (0)
// lean kernel: absolute shader-clock stamps per document (no atomics): ygm_diag_ts[(d % 16384) * 8 + slot]
__device__ unsigned long long ygm_diag_ts[16384 * 8];
// (s_memrealtime: the chip-wide 100 MHz clock, comparable across waves and XCDs)
#define DIAGL_T0 if (threadIdx.x == 0) ygm_diag_ts[(blockIdx.x & 16383u) * 8] = __builtin_amdgcn_s_memrealtime();
#define DIAGL(i) do { if (threadIdx.x == 0) ygm_diag_ts[(blockIdx.x & 16383u) * 8 + 1 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define DIAG_NOW() __builtin_amdgcn_s_memrealtime()
#define DIAG_PUT(i, v) do { if (threadIdx.x == 0) ygm_diag_ts[(blockIdx.x & 16383u) * 8 + (i)] = (v); } while (0)
#define DIAG_C(...) __VA_ARGS__
#else
#define DIAGL_T0
#define DIAGL(i)
#define DIAG_NOW() 0ull
#define DIAG_PUT(i, v)
#define DIAG_C(...)
#define DIAGW(i)
#define DIAG_T0
#define DIAG(i)
#endif

namespace ygm {

// ======================================================================= SV / diff
constexpr int DOC_NT = 256;   // lanes (= documents) per workgroup tile
constexpr int DIFF_BLK = 16;  // per-lane LDS slots for output-block counts

YDEV uint64_t merge_place(const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t d, uint64_t size, uint64_t slot_total,
                          DocMeta* meta) {
  const uint64_t b0 = upd_off[doc_upd[d]], b1 = upd_off[doc_upd[d + 1]];
  if (size <= merge_slot_cap(b1 - b0)) return merge_slot(b0, d);
  return slot_total + atomicAdd(&meta->cursor, (unsigned long long)size);
}

template <int MODE>  // 0 = sv, 1 = diff
__global__ __launch_bounds__(DOC_NT) void k_doc(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off,
                                                 const uint8_t* __restrict__ sv_arena, const uint64_t* __restrict__ sv_off,
                                                 const uint32_t* __restrict__ docs, uint64_t out_base,
                                                 uint32_t n_docs, uint32_t flags, uint8_t* __restrict__ out,
                                                 uint64_t* __restrict__ out_off, uint64_t* __restrict__ out_len,
                                                 int32_t* __restrict__ status, unsigned long long* lb, DocMeta* meta,
                                                 uint64_t out_cap) {
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_tmp[DOC_NT / WAVE + 1];
  __shared__ uint64_t s_base;
  __shared__ uint32_t s_blk[MODE == 1 ? DOC_NT * DIFF_BLK : 1];
  if (threadIdx.x == 0) s_tile = atomicAdd(&meta->ticket, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t di = tile * DOC_NT + threadIdx.x;   // index into `docs` (the lean kernel's deferred list) or the document
  const bool live = di < n_docs;
  const uint32_t d = live ? (docs ? docs[di] : di) : 0u;
  const uint8_t* p = nullptr; uint32_t n = 0;
  const uint8_t* sv = nullptr; uint32_t svn = 0;
  if (live) {
    const uint64_t a = doc_off[d], b = doc_off[d + 1];
    p = arena + a; n = (uint32_t)(b - a);
    if (MODE == 1) { const uint64_t sa = sv_off[d], sb = sv_off[d + 1]; sv = sv_arena + sa; svn = (uint32_t)(sb - sa); }
  }
  uint32_t* blk = &s_blk[MODE == 1 ? threadIdx.x * DIFF_BLK : 0];
  int st = ST_OK; uint64_t aux = 0;
  Out o{nullptr, 0};
  if (live) {
    if (MODE == 0) st = sv_doc(p, n, flags, o, aux, false);
    else st = diff_doc(p, n, sv, svn, flags, o, false, aux, blk, DIFF_BLK);
  }
  const uint64_t mysz = (live && st == ST_OK) ? o.n : 0;
  uint64_t tot;
  const uint64_t pre = block_exscan<DOC_NT>(mysz, s_tmp, tot);
  if (threadIdx.x < WAVE) {
    const uint64_t b = lookback(lb, tile, tot, &meta->fault);
    if (threadIdx.x == 0) {
      s_base = b;
      if (tile == (n_docs - 1) / DOC_NT) meta->fast_total = b + tot;
    }
  }
  __syncthreads();
  if (!live) return;
  const uint64_t at = out_base + s_base + pre;
  if (st == ST_OK && at + mysz > out_cap) st = ST_NOMEM;
  if (st == ST_OK) {
    Out w{out + at, 0};
    const int e = MODE == 0 ? sv_doc(p, n, flags, w, aux, true) : diff_doc(p, n, sv, svn, flags, w, true, aux, blk, DIFF_BLK);
    if (e) st = e;
  }
  if (meta->fault) st = ST_DEVICE;
  out_off[d] = at; out_len[d] = st == ST_OK ? mysz : 0; status[d] = st;
}


// ======================================================================= merge fast path
// LDS capacity of one document (class "small").  Documents beyond any of these
// take the sequential kernel.
constexpr int M_NT = 256;
constexpr int M_KCAP = 256;      // updates
constexpr int M_INCAP = 16384;   // input bytes
constexpr int M_SCAP = 512;      // structs (non-Skip)
constexpr int M_DCAP = 256;      // delete-set ranges

struct MergeLds {
  uint8_t in[M_INCAP + 16];
  uint32_t ustart[M_KCAP], ulen[M_KCAP], uns[M_KCAP], und[M_KCAP];
  uint64_t key[M_SCAP];
  uint16_t idx[M_SCAP];
  uint32_t r_start[M_SCAP], r_len[M_SCAP], r_out[M_SCAP];
  uint16_t r_src[M_SCAP], r_seq[M_SCAP];
  uint8_t r_kind[M_SCAP];
  uint32_t eF[M_SCAP], eA[M_SCAP], eB[M_SCAP], eC[M_SCAP], eE[M_SCAP];
  uint64_t dkey[M_DCAP];
  uint16_t didx[M_DCAP];
  uint32_t d_len[M_DCAP];
  uint64_t dA[M_DCAP];
  uint32_t dB[M_DCAP], dC[M_DCAP], dE[M_DCAP], dF[M_DCAP];
  uint32_t d_cl[M_DCAP], d_rk[M_DCAP];   // by record: client; first-seen rank (update << 16 | range in it: yjs 13.5)
  uint64_t tmp64[M_NT / WAVE + 1];
  uint32_t tmp32[M_NT / WAVE + 1];
  int err, fb, nc;
  uint32_t tile, nseg;
  uint64_t base;
};

enum : uint32_t {  // eF bits (per sorted struct)
  EF_NEWC = 1, EF_GAP = 2, EF_CGG = 4, EF_SDN = 8, EF_T = 16, EF_GC = 32, EF_EMIT = 64, EF_NONID = 128
};

// parse update i of the staged document: pass 0 counts, pass 1 fills records
YDEV_NI void m_parse_update(MergeLds& L, int i, int pass, uint32_t flags) {
  Cur c{L.in, L.ustart[i], L.ustart[i] + L.ulen[i], 0, 0};
  uint32_t s_at = pass ? L.uns[i] : 0, d_at = pass ? L.und[i] : 0;
  uint32_t ns = 0, nd = 0; bool fb = false, nc = false;
  uint64_t prev_client = 0, prev_end = 0; bool have_prev = false;
  const uint64_t nb = c.vu();
  for (uint64_t b = 0; b < nb && !c.err; b++) {
    const uint64_t nst = c.vu(), client = c.vu(); uint64_t clock = c.vu();
    if (c.err) break;
    if (client > 0xFFFFFFFFull) fb = true;
    for (uint64_t s = 0; s < nst && !c.err; s++) {
      SInfo si; read_struct_fast<true>(c, si, flags);   // (the cursor stays in registers)
      if (c.err) break;
      const uint64_t end = clock + si.len;
      if (end > MAX_SAFE) { c.fail(ST_RANGE); break; }
      if (si.kind != K_SKIP) {
        if (si.len == 0 || end > 0xFFFFFFFFull) fb = true;
        // sequence must be sorted (client desc, clock asc) and overlap-free
        if (have_prev && (client > prev_client || (client == prev_client && clock < prev_end))) fb = true;
        have_prev = true; prev_client = client; prev_end = end;
        if (si.nc) nc = true;
        if (pass && !fb && s_at + ns < M_SCAP) {
          const uint32_t j = s_at + ns;
          L.key[j] = ((uint64_t)(0xFFFFFFFFu - (uint32_t)client) << 32) | (uint32_t)clock;
          L.idx[j] = (uint16_t)j;
          L.r_start[j] = si.start; L.r_len[j] = (uint32_t)si.len;
          L.r_src[j] = (uint16_t)i; L.r_seq[j] = (uint16_t)ns;
          L.r_kind[j] = (uint8_t)si.kind;
          if (si.kind == K_ITEM) { Out o{nullptr, 0}; write_struct(o, L.in, si, client, clock, 0, false, flags); L.r_out[j] = o.n; }
          else L.r_out[j] = 0;
        }
        ns++;
      }
      clock = end;
    }
  }
  // delete set
  const uint64_t ncl = c.err ? 0 : c.vu();
  for (uint64_t q = 0; q < ncl && !c.err; q++) {
    const uint64_t cl = c.vu(), nr = c.vu();
    for (uint64_t r = 0; r < nr && !c.err; r++) {
      const uint64_t ck = c.vu(), ln = c.vu();
      if (c.err) break;
      if (cl > 0xFFFFFFFFull || ck + ln > 0xFFFFFFFFull) fb = true;
      if (pass && !fb && d_at + nd < M_DCAP) {
        const uint32_t j = d_at + nd;
        L.dkey[j] = ((uint64_t)(0xFFFFFFFFu - (uint32_t)cl) << 32) | (uint32_t)ck;
        L.didx[j] = (uint16_t)j; L.d_len[j] = (uint32_t)ln;
        L.d_cl[j] = (uint32_t)cl; L.d_rk[j] = ((uint32_t)i << 16) | (uint32_t)nd;
      }
      nd++;
    }
  }
  if (c.err) { atomicCAS(&L.err, 0, c.err); return; }
  if (fb) atomicOr(&L.fb, 1);
  if (nc) atomicOr(&L.nc, 1);
  if (!pass) { L.uns[i] = ns; L.und[i] = nd; }
}

YDEV int pow2_ceil(int n) { int p = 1; while (p < n) p <<= 1; return p; }

// Documents deferred by the wave kernel (list `docs`, n_docs entries), one
// workgroup each; outputs placed by merge_place.
YDEV void merge_fast_doc(MergeLds& L, uint32_t d, const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                         const uint32_t* __restrict__ doc_upd, uint32_t flags,
                         uint8_t* __restrict__ out_all, uint64_t* __restrict__ out_off,
                         uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                         uint64_t slot_total, DocMeta* meta, uint32_t* fb_list, uint64_t out_cap) {
  const int t = threadIdx.x;
  DIAG_T0
  if (t == 0) { L.err = 0; L.fb = 0; L.nc = 0; }
  __syncthreads();
  const uint32_t u0 = doc_upd[d], u1 = doc_upd[d + 1];
  const uint32_t k = u1 - u0;
  const uint64_t b0 = upd_off[u0], b1 = upd_off[u1];
  const uint64_t nbytes = b1 - b0;
  int st = ST_OK;
  uint64_t size = 0;
  int mode = 0;  // 0 merge, 1 empty "0000", 2 passthrough (single input, Y@39011)
  int S = 0, D = 0; uint32_t nblocks = 0, hdr0 = 0, struct_bytes = 0;
  if (k == 0) { mode = 1; size = 2; }
  else if (k == 1) { mode = 2; size = nbytes; }
  else if (k > (uint32_t)M_KCAP || nbytes > (uint64_t)M_INCAP || (flags & 2u /*YGM_F_FORCE_SEQ*/)) st = ST_FALLBACK;
  if (mode == 0 && st == ST_OK) {
    // ---- stage the document's bytes into LDS (coalesced) and the update table
    for (uint32_t i = t; i < (uint32_t)nbytes; i += M_NT) L.in[i] = arena[b0 + i];
    for (uint32_t i = t; i < k; i += M_NT) { const uint64_t a = upd_off[u0 + i], b = upd_off[u0 + i + 1]; L.ustart[i] = (uint32_t)(a - b0); L.ulen[i] = (uint32_t)(b - a); }
    __syncthreads();
    DIAG(0);
    // ---- pass A: validate + count
    for (uint32_t i = t; i < k; i += M_NT) m_parse_update(L, i, 0, flags);
    __syncthreads();
    DIAG(1);
    if (L.err) st = L.err;
    else if (L.fb) st = ST_FALLBACK;
    if (st == ST_OK) {
      S = (int)block_scan_array<M_NT>(L.uns, (int)k, L.tmp32);
      D = (int)block_scan_array<M_NT>(L.und, (int)k, L.tmp32);
      if (S > M_SCAP || D > M_DCAP) st = ST_FALLBACK;
      else if (L.nc) st = ST_NONCANON;
    }
  }
  if (mode == 0 && st == ST_OK) {
    // ---- pass B: records
    for (uint32_t i = t; i < k; i += M_NT) m_parse_update(L, i, 1, flags);
    const int NS = pow2_ceil(S > 0 ? S : 1), ND = pow2_ceil(D > 0 ? D : 1);
    for (int j = S + t; j < NS; j += M_NT) { L.key[j] = ~0ull; L.idx[j] = 0xFFFF; }
    for (int j = D + t; j < ND; j += M_NT) { L.dkey[j] = ~0ull; L.didx[j] = 0xFFFF; }
    __syncthreads();
    if (flags & F_COMPAT_135) {
      // yjs 13.5 writes the merged delete set's clients in first-seen order (mergeDeleteSets' Map insertion order,
      // Y@10486): a client's key is its least record rank instead of its complement, so the sort groups its ranges
      // in that order (ranks of different clients differ; the client itself is read from d_cl)
      for (int j = t; j < D; j += M_NT) {
        const uint32_t c = L.d_cl[j];
        uint32_t r = L.d_rk[j];
        for (int q = 0; q < D; q++) if (L.d_cl[q] == c && L.d_rk[q] < r) r = L.d_rk[q];
        L.dkey[j] = ((uint64_t)r << 32) | (uint32_t)L.dkey[j];
      }
      __syncthreads();
    }
    DIAG(2);
    bitonic_sort<M_NT>(L.key, L.idx, NS);
    bitonic_sort<M_NT>(L.dkey, L.didx, ND);
    DIAG(3);
    // ---- structs: classify each sorted element against its predecessor
    for (int j = t; j < S; j += M_NT) {
      const uint64_t kj = L.key[j]; const uint32_t r = L.idx[j];
      const uint32_t cl = (uint32_t)(kj >> 32), ck = (uint32_t)kj;
      uint32_t f = (L.r_kind[r] == K_GC) ? EF_GC : 0;
      if (j == 0) f |= EF_NEWC;
      else {
        const uint64_t kp = L.key[j - 1]; const uint32_t rp = L.idx[j - 1];
        const uint32_t pend = (uint32_t)kp + L.r_len[rp];
        if ((uint32_t)(kp >> 32) != cl) f |= EF_NEWC;
        else if (ck < pend) atomicOr(&L.fb, 1);           // overlap -> exact sequential replay
        else if (ck > pend) f |= EF_GAP;
        else {
          if (L.r_src[r] == L.r_src[rp] && L.r_seq[r] == L.r_seq[rp] + 1) f |= EF_SDN;
          if ((f & EF_GC) && L.r_kind[rp] == K_GC) f |= EF_CGG;
        }
      }
      // transfer function of the GC-merge state (last write was "new struct")
      if (!(f & EF_CGG)) f |= EF_NONID | EF_T;
      else if (!(f & EF_SDN)) f |= EF_NONID;
      L.eF[j] = f;
      L.eA[j] = (f & EF_NONID) ? (uint32_t)(j + 1) : 0u;
      L.eB[j] = (f & EF_NEWC) ? 1u : 0u;
      L.eC[j] = 0;
    }
    __syncthreads();
    if (L.fb) st = ST_FALLBACK;
  }
  if (mode == 0 && st == ST_OK) {
    block_maxscan_array<M_NT>(L.eA, S, L.tmp32, 0u);
    nblocks = block_scan_array<M_NT>(L.eB, S, L.tmp32);  // eB[j] = #NEWC before j
    for (int j = t; j < S; j += M_NT) {
      const uint32_t lnid = L.eA[j] - 1;                  // last non-identity element <= j
      const bool last_new = (L.eF[lnid] & EF_T) != 0;
      if (last_new) L.eF[j] |= EF_EMIT;                   // else merged into the previous GC
    }
    __syncthreads();
    // block index: eB is the exclusive count of NEWC, so element j belongs to block eB[j] + NEWC(j) - 1
    for (int j = t; j < S; j += M_NT) {
      const uint32_t f = L.eF[j];
      const uint32_t blk = L.eB[j] + ((f & EF_NEWC) ? 1u : 0u) - 1u;
      L.eB[j] = blk;
      const uint32_t cnt = ((f & EF_GAP) ? 1u : 0u) + ((f & EF_EMIT) ? 1u : 0u);
      atomicAdd(&L.eC[blk], cnt);
      L.eA[j] = (f & EF_EMIT) ? (uint32_t)(j + 1) : 0u;  // for GC run heads
      L.eE[j] = (uint32_t)L.key[j] + L.r_len[L.idx[j]];   // end
    }
    __syncthreads();
    block_maxscan_array<M_NT>(L.eA, S, L.tmp32, 0u);
    for (int j = t; j < S; j += M_NT) {
      if (!(L.eF[j] & EF_EMIT)) { const uint32_t head = L.eA[j] - 1; atomicMax(&L.eE[head], L.eE[j]); }
    }
    __syncthreads();
    // element sizes -> eA
    for (int j = t; j < S; j += M_NT) {
      const uint32_t f = L.eF[j]; const uint64_t kj = L.key[j]; const uint32_t r = L.idx[j];
      const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(kj >> 32), ck = (uint32_t)kj;
      uint32_t sz = 0;
      if (f & EF_NEWC) sz += vu_len(L.eC[L.eB[j]]) + vu_len(cl) + vu_len(ck);
      if (f & EF_GAP) { const uint64_t kp = L.key[j - 1]; const uint32_t pend = (uint32_t)kp + L.r_len[L.idx[j - 1]]; sz += 1 + vu_len(ck - pend); }
      if (f & EF_EMIT) sz += (f & EF_GC) ? 1 + vu_len(L.eE[j] - ck) : L.r_out[r];
      L.eA[j] = sz;
    }
    __syncthreads();
    struct_bytes = block_scan_array<M_NT>(L.eA, S, L.tmp32);
    hdr0 = vu_len(nblocks);
    DIAG(4);
    // ---- delete set: segments (clients) and runs
    for (int j = t; j < D; j += M_NT) {
      const uint64_t kj = L.dkey[j];
      const bool segnew = j == 0 || (L.dkey[j - 1] >> 32) != (kj >> 32);
      L.dB[j] = segnew ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t nseg = block_scan_array<M_NT>(L.dB, D, L.tmp32);  // dB[j] = #segments before j
    for (int j = t; j < D; j += M_NT) {
      const uint64_t kj = L.dkey[j];
      const bool segnew = j == 0 || (L.dkey[j - 1] >> 32) != (kj >> 32);
      const uint32_t seg = L.dB[j] + (segnew ? 1u : 0u) - 1u;
      L.dB[j] = seg;
      L.dA[j] = ((uint64_t)seg << 32) | ((uint32_t)kj + L.d_len[L.didx[j]]);
      L.dC[j] = 0; L.dE[j] = 0;
    }
    __syncthreads();
    block_maxscan_array<M_NT>(L.dA, D, L.tmp64, (uint64_t)0);
    // run starts: new segment, or clock beyond the running end of the segment
    for (int j = t; j < D; j += M_NT) {
      const uint32_t ck = (uint32_t)L.dkey[j];
      const bool segnew = j == 0 || L.dB[j - 1] != L.dB[j];
      const bool rs = segnew || ck > (uint32_t)L.dA[j - 1];
      L.dF[j] = (segnew ? 1u : 0u) | (rs ? 2u : 0u);
      if (rs) atomicAdd(&L.dC[L.dB[j]], 1u);             // runs per segment
    }
    __syncthreads();
    // run end = running max at the run's last element
    for (int j = t; j < D; j += M_NT) {
      const bool last = j == D - 1 || (L.dF[j + 1] & 2u);
      if (last) {
        int s = j; while (!(L.dF[s] & 2u)) s--;          // walk back to the run start (runs are short)
        L.dE[s] = (uint32_t)L.dA[j];
      }
    }
    __syncthreads();
    for (int j = t; j < D; j += M_NT) {
      const uint32_t f = L.dF[j]; const uint64_t kj = L.dkey[j];
      const uint32_t cl = L.d_cl[L.didx[j]], ck = (uint32_t)kj;
      uint32_t sz = 0;
      if (f & 1u) sz += vu_len(cl) + vu_len(L.dC[L.dB[j]]);
      if (f & 2u) sz += vu_len(ck) + vu_len(L.dE[j] - ck);
      L.dA[j] = sz;
    }
    __syncthreads();
    const uint64_t ds_bytes = block_scan_array<M_NT>(L.dA, D, L.tmp64) + vu_len(nseg);
    size = hdr0 + struct_bytes + ds_bytes;
    if (t == 0) L.nseg = nseg;
  }
  DIAG(5);
  // ---- placement: the document's own slot (or the overflow region)
  if (t == 0) {
    L.base = st == ST_OK ? merge_place(upd_off, doc_upd, d, size, slot_total, meta) : 0;
    if (st == ST_FALLBACK) {
      const uint32_t q = atomicAdd(&meta->fb_count, 1u);
      fb_list[q] = d;
      atomicAdd(&meta->fb_upds, (unsigned long long)k);
      atomicAdd(&meta->fb_bytes, (unsigned long long)nbytes);
    }
  }
  __syncthreads();
  DIAG(6);
  const uint64_t base = L.base;
  if (st == ST_OK && base + size > out_cap) st = ST_NOMEM;
  if (t == 0) {
    if (st == ST_OK) add_payload(meta, d, size);
    out_off[d] = base; out_len[d] = st == ST_OK ? size : 0; status[d] = st;
  }
  if (st != ST_OK) return;
  uint8_t* o = out_all + base;
  if (mode == 1) { if (t == 0) { o[0] = 0; o[1] = 0; } return; }
  if (mode == 2) { for (uint64_t i = t; i < nbytes; i += M_NT) o[i] = arena[b0 + i]; return; }
  // ---- emit structs
  if (t == 0) { Out w{o, 0}; w.vu(nblocks); }
  for (int j = t; j < S; j += M_NT) {
    const uint32_t f = L.eF[j]; const uint64_t kj = L.key[j]; const uint32_t r = L.idx[j];
    const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(kj >> 32), ck = (uint32_t)kj;
    Out w{o + hdr0 + L.eA[j], 0};
    if (f & EF_NEWC) { w.vu(L.eC[L.eB[j]]); w.vu(cl); w.vu(ck); }
    if (f & EF_GAP) { const uint64_t kp = L.key[j - 1]; const uint32_t pend = (uint32_t)kp + L.r_len[L.idx[j - 1]]; w.b(10); w.vu(ck - pend); }
    if (f & EF_EMIT) {
      if (f & EF_GC) { w.b(0); w.vu(L.eE[j] - ck); }
      else { Cur c{L.in, L.r_start[r], L.ustart[L.r_src[r]] + L.ulen[L.r_src[r]], 0, 0}; SInfo si; read_struct<true>(c, si, flags); write_struct(w, L.in, si, cl, ck, 0, false, flags); }
    }
  }
  // ---- emit delete set
  const uint32_t dsb = hdr0 + struct_bytes;
  if (t == 0) { Out w{o + dsb, 0}; w.vu(L.nseg); }
  const uint32_t dh = vu_len(L.nseg);
  for (int j = t; j < D; j += M_NT) {
    const uint32_t f = L.dF[j]; const uint64_t kj = L.dkey[j];
    const uint32_t cl = L.d_cl[L.didx[j]], ck = (uint32_t)kj;
    Out w{o + dsb + dh + (uint32_t)L.dA[j], 0};
    if (f & 1u) { w.vu(cl); w.vu(L.dC[L.dB[j]]); }
    if (f & 2u) { w.vu(ck); w.vu(L.dE[j] - ck); }
  }
  DIAG(7);
}

// Documents deferred by the wave kernel, one workgroup at a time (persistent grid).  The count is
// read from device memory (`n_dev`, written by the previous kernel in stream order) when given.
__global__ __launch_bounds__(M_NT) void k_merge_fast(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                      const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ docs,
                                                      const unsigned int* n_dev, uint32_t n_docs, uint32_t flags,
                                                      uint8_t* __restrict__ out_all, uint64_t* __restrict__ out_off,
                                                      uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                                                      uint64_t slot_total, DocMeta* meta, uint32_t* fb_list, uint64_t out_cap) {
  __shared__ MergeLds L;
  const uint32_t N = n_dev ? *n_dev : n_docs;
  for (uint32_t i = blockIdx.x; i < N; i += gridDim.x) {
    merge_fast_doc(L, docs[i], arena, upd_off, doc_upd, flags, out_all, out_off, out_len, status, slot_total, meta, fb_list, out_cap);
    __syncthreads();
  }
}


// ======================================================================= merge: one wave per document
// See ygm_merge_wave.hpp for the phase plan.  Per-element state lives in LDS
// and every per-element loop is rolled (the kernel stays I-cache sized).
YDEV uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) { const uint32_t o = (uint32_t)__shfl_xor((int)v, d, WAVE); v = o < v ? o : v; }
  return v;
}

#ifndef YGM_BIG_ROUTE
#define YGM_BIG_ROUTE 1024
#endif
constexpr uint32_t BIG_ROUTE_MIN = YGM_BIG_ROUTE;   // snapshot bytes from which a document goes to k_merge_big directly
YDEV void merge_wave_doc(WaveLds& L, uint32_t d, const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                         const uint32_t* __restrict__ doc_upd, uint32_t flags,
                         uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                         uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                         DocMeta* meta, uint32_t* defer_list, uint32_t* fb_list, uint64_t out_cap) {
  DIAG_T0
  const uint32_t l = threadIdx.x % WAVE;
  LWave* LW = (LWave*)&L;
  const uint32_t u0 = doc_upd[d], u1 = doc_upd[d + 1];
  const uint32_t k = u1 - u0;
  const uint64_t b0 = upd_off[u0], b1 = upd_off[u1];
  const uint64_t nbytes = b1 - b0;
  const uint64_t slot = merge_slot(b0, d), cap = merge_slot_cap(nbytes);
  constexpr int ST_DEFER = 101;
  int st = ST_OK, mode = 0;
  uint64_t size = 0;
  uint32_t S = 0, D = 0, nC = 0, nseg = 0, hdr0 = 0, sbytes = 0, dsbytes = 0;
  if (k == 0) { mode = 1; size = 2; }
  else if (k == 1) { mode = 2; size = nbytes; }
  else if (flags & 2u) st = ST_DEFER;
  else {
    // [snapshot, ...log] documents whose snapshot is large go straight to the large-document tier: its
    // parallel walk of the snapshot beats the lane-per-update parse of this kernel and of the workgroup
    // tier, which walk the snapshot on one lane
    uint64_t mx = 0;
    for (uint32_t i = l; i < k; i += WAVE) { const uint64_t n = upd_off[u0 + i + 1] - upd_off[u0 + i]; mx = n > mx ? n : mx; }
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) { const uint64_t t = __shfl_xor(mx, o, WAVE); mx = t > mx ? t : mx; }
    if (mx >= (uint64_t)BIG_ROUTE_MIN) st = ST_FALLBACK;
    else if (k > (uint32_t)W_K || nbytes + 16 > (uint64_t)W_IN) st = ST_DEFER;
  }
  if (mode == 0 && st == ST_OK) {
    // ---- stage: 16-byte loads of [b0 & ~15, b1) (arenas carry >= 16 readable bytes of tail padding)
    const uint64_t a0 = b0 & ~15ull;
    const uint32_t shift = (uint32_t)(b0 - a0);
    const uint32_t nch = (uint32_t)((shift + nbytes + 15) / 16);
    for (uint32_t c = l; c < nch; c += WAVE) *(uint4*)(L.in + c * 16) = *(const uint4*)(arena + a0 + (uint64_t)c * 16);
    for (uint32_t i = l; i < k; i += WAVE) {
      const uint64_t a = upd_off[u0 + i], b = upd_off[u0 + i + 1];
      L.ustart[i] = (uint16_t)(a - b0 + shift); L.ulen[i] = (uint16_t)(b - a);
    }
    if (l == 0) { L.nrec = 0; L.ndel = 0; }
    wave_sync();
    DIAGW(0);
    // ---- parse: one pass, lane l takes updates l, l+64, ...; first error by update index wins
    uint32_t ekey = 0xFFFFFFFFu; bool fb = false, nc = false;
    for (uint32_t i = l; i < k; i += WAVE) {
      const UpdCount c = w_parse_update(LW, (int)i, flags);
      fb |= c.fb != 0; nc |= c.nc != 0;
      if (c.err) { ekey = (i << 8) | (uint32_t)c.err; break; }
    }
    wave_sync();
    DIAGW(1);
    ekey = wave_min_u32(ekey);
    S = L.nrec; D = L.ndel;
    if (ekey != 0xFFFFFFFFu) st = (int)(ekey & 0xFF);
    else if (__ballot(fb) || S > (uint32_t)W_S || D > (uint32_t)W_D) st = ST_DEFER;
    else if (__ballot(nc)) st = ST_NONCANON;
    if (st == ST_OK) {
      // ---- clients: distinct values by wave vote, ranked descending
      uint32_t rc[W_E]; uint8_t cid[W_E];
#pragma unroll
      for (int q = 0; q < W_E; q++) { const uint32_t e = l + WAVE * q; rc[q] = e < S ? L.rcl[e] : 0; cid[q] = e < S ? 0xFF : 0xFE; }
      uint32_t myc = 0;
      for (;;) {
        bool has = false; uint32_t cand = 0;
#pragma unroll
        for (int q = 0; q < W_E; q++) if (cid[q] == 0xFF && !has) { has = true; cand = rc[q]; }
        const uint64_t m = __ballot(has);
        if (!m) break;
        if (nC == (uint32_t)W_C) { st = ST_DEFER; break; }
        const uint32_t c = (uint32_t)__shfl((int)cand, __ffsll((long long)m) - 1, WAVE);
#pragma unroll
        for (int q = 0; q < W_E; q++) if (cid[q] == 0xFF && rc[q] == c) cid[q] = (uint8_t)nC;
        if (l == nC) myc = c;
        nC++;
      }
      if (st == ST_OK) {
        uint32_t rank = 0;
        for (uint32_t t = 0; t < nC; t++) rank += (uint32_t)__shfl((int)myc, (int)t, WAVE) > myc ? 1u : 0u;
        if (l < nC) { L.ctab[rank] = myc; L.blkcnt[rank] = 0; }
        // ---- sort keys (client rank << 40 | clock << 8 | record) in registers
        uint64_t kr[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t e = l + WAVE * q;
          const uint32_t cr = (uint32_t)__shfl((int)rank, q < W_E ? (int)(cid[q] & 63) : 0, WAVE);
          kr[q] = (q < W_E && e < S) ? (L.key[e] | ((uint64_t)cr << 40)) : ~0ull;
        }
        // stable split by client rank (records were allocated in update order, so a
        // log whose updates arrive in clock order per client is sorted after it);
        // anything else: bitonic sort
        bool sorted = false;
        if (nC <= 8) {
          uint32_t pos[W_E], base = 0;
          for (uint32_t b = 0; b < nC; b++) {
#pragma unroll
            for (int q = 0; q < W_E; q++) {
              const bool in_b = (kr[q] >> 40) == b;   // padding keys (~0) never match
              const uint64_t m = __ballot(in_b);
              if (in_b) pos[q] = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
              base += (uint32_t)__popcll(m);
            }
          }
#pragma unroll
          for (int q = 0; q < W_E; q++) if (l + WAVE * q < S) L.key[pos[q]] = kr[q];
          wave_sync();
          bool bad = false;
          for (uint32_t j = l + 1; j < S; j += WAVE) bad |= L.key[j - 1] > L.key[j];
          sorted = __ballot(bad) == 0;
          wave_sync();
        }
        if (!sorted) {
          if (S <= 64) wave_bitonic<1>(kr);
          else if (S <= 128) wave_bitonic<2>(kr);
          else wave_bitonic<4>(kr);
          const uint32_t E = S <= 64 ? 1u : S <= 128 ? 2u : 4u;
#pragma unroll
          for (int q = 0; q < 4; q++) { const uint32_t i = E * l + q; if ((uint32_t)q < E && i < S) L.key[i] = kr[q]; }
        }
        for (uint32_t j = l; j < S; j += WAVE) L.rcl[j] = 0;   // becomes the GC run end by sorted element
        wave_sync();
        DIAGW(2);
        // ---- classify sorted structs (blocked: lane l owns elements l*W_E .. l*W_E+W_E-1)
        const uint32_t e0 = l * W_E, e1 = min(e0 + W_E, S);
        bool ovl = false;
        uint32_t vmax = 0;
        for (uint32_t j = e0; j < e1; j++) {
          const uint64_t kj = L.key[j]; const uint32_t r = (uint32_t)kj & 0xFF;
          const uint32_t rbj = L.rb[r];
          uint32_t f = ((rbj >> 13) & 3) == K_GC ? EF_GC : 0;
          if (j == 0 || (L.key[j - 1] >> 40) != (kj >> 40)) f |= EF_NEWC;
          else {
            const uint64_t kp = L.key[j - 1]; const uint32_t rp = (uint32_t)kp & 0xFF;
            const uint32_t pend = (uint32_t)(kp >> 8) + (uint32_t)L.ra[rp];
            const uint32_t ck = (uint32_t)(kj >> 8);
            const uint32_t rbp = L.rb[rp];
            if (ck < pend) ovl = true;
            else if (ck > pend) f |= EF_GAP;
            else {
              const uint32_t ss = rbj >> 16, sp = rbp >> 16;
              if ((ss >> 8) == (sp >> 8) && (ss & 0xFF) == (sp & 0xFF) + 1) f |= EF_SDN;
              if ((f & EF_GC) && ((rbp >> 13) & 3) == K_GC) f |= EF_CGG;
            }
          }
          if (!(f & EF_CGG)) f |= EF_NONID | EF_T;
          else if (!(f & EF_SDN)) f |= EF_NONID;
          L.eflag[j] = (uint8_t)f;
          if (f & EF_NONID) vmax = j + 1;
        }
        if (__ballot(ovl)) st = ST_FALLBACK;  // overlapping structs: exact sequential replay
        else {
          wave_sync();
          // GC provenance: last non-identity element <= j (max-scan); emitted heads
          uint32_t mex = wave_incl_scan_max(vmax); mex = __shfl_up(mex, 1, WAVE); if (l == 0) mex = 0;
          uint32_t hmax = 0, lastnid = mex;
          for (uint32_t j = e0; j < e1; j++) {
            uint32_t f = L.eflag[j];
            if (f & EF_NONID) lastnid = j + 1;
            if (L.eflag[lastnid - 1] & EF_T) f |= EF_EMIT;   // otherwise merged into the previous GC
            L.eflag[j] = (uint8_t)f;
            if (f & EF_EMIT) hmax = j + 1;
          }
          uint32_t hex = wave_incl_scan_max(hmax); hex = __shfl_up(hex, 1, WAVE); if (l == 0) hex = 0;
          // per-client struct counts, GC run ends (LDS atomics)
          uint32_t head = hex;
          for (uint32_t j = e0; j < e1; j++) {
            const uint32_t f = L.eflag[j];
            const uint64_t kj = L.key[j];
            if (f & EF_EMIT) head = j + 1;
            const uint32_t cnt = ((f & EF_GAP) ? 1u : 0u) + ((f & EF_EMIT) ? 1u : 0u);
            if (cnt) atomicAdd(&L.blkcnt[kj >> 40], cnt);
            atomicMax(&L.rcl[head - 1], (uint32_t)(kj >> 8) + (uint32_t)L.ra[kj & 0xFF]);
          }
          wave_sync();
          // element sizes -> positions (epos, relative to the struct section)
          uint32_t acc = 0;
          for (uint32_t j = e0; j < e1; j++) {
            const uint32_t f = L.eflag[j];
            const uint64_t kj = L.key[j]; const uint32_t r = (uint32_t)kj & 0xFF;
            const uint32_t crk = (uint32_t)(kj >> 40), ck = (uint32_t)(kj >> 8);
            uint32_t sz = 0;
            if (f & EF_NEWC) sz += vu_len(L.blkcnt[crk]) + vu_len(L.ctab[crk]) + vu_len(ck);
            if (f & EF_GAP) { const uint64_t kp = L.key[j - 1]; sz += 1 + vu_len(ck - ((uint32_t)(kp >> 8) + (uint32_t)L.ra[kp & 0xFF])); }
            if (f & EF_EMIT) sz += (f & EF_GC) ? 1 + vu_len(L.rcl[j] - ck) : (L.rb[r] & 0x1FFF);
            L.epos[j] = (uint16_t)acc; acc += sz;
          }
          const uint32_t lb0 = wave_exscan(acc, sbytes);
          for (uint32_t j = e0; j < e1; j++) L.epos[j] = (uint16_t)(L.epos[j] + lb0);
          hdr0 = vu_len(nC);
          DIAGW(3);
          // ---- delete set: rank sort, segments (clients, descending) and runs (rule R-DS)
          if (D) {
            uint64_t mk[W_DE]; uint32_t ml[W_DE], rk[W_DE], mc[W_DE];
#pragma unroll
            for (int q = 0; q < W_DE; q++) {
              const uint32_t j = l + WAVE * q;
              mk[q] = j < D ? L.dkey[j] : ~0ull; ml[q] = j < D ? L.dlen[j] : 0; rk[q] = 0; mc[q] = j < D ? L.dcl[j] : 0;
            }
            if (flags & F_COMPAT_135) {
              // yjs 13.5: the merged delete set's clients in first-seen order (Y@10486) -- a client's key is its least
              // record rank (update << 8 | range in it, parked in drunend by the parse) instead of its complement
#pragma unroll
              for (int q = 0; q < W_DE; q++) {
                uint32_t r = l + WAVE * q < D ? L.drunend[l + WAVE * q] : 0u;
                for (uint32_t i = 0; i < D; i++) {
                  const uint32_t ri = L.drunend[i];
                  r = L.dcl[i] == mc[q] && ri < r ? ri : r;
                }
                if (l + WAVE * q < D) mk[q] = ((uint64_t)r << 32) | (uint32_t)mk[q];
              }
              wave_sync();
#pragma unroll
              for (int q = 0; q < W_DE; q++) if (l + WAVE * q < D) L.dkey[l + WAVE * q] = mk[q];
              wave_sync();
            }
            for (uint32_t i = 0; i < D; i++) {
              const uint64_t ki = L.dkey[i];
#pragma unroll
              for (int q = 0; q < W_DE; q++) rk[q] += (ki < mk[q]) || (ki == mk[q] && i < l + WAVE * q);
            }
            wave_sync();
#pragma unroll
            for (int q = 0; q < W_DE; q++) if (l + WAVE * q < D) { L.dkey[rk[q]] = mk[q]; L.dlen[rk[q]] = ml[q]; L.dcl[rk[q]] = mc[q]; }
            for (uint32_t j = l; j < D; j += WAVE) L.drunend[j] = 0;
            for (uint32_t j = l; j < W_BLK; j += WAVE) L.segcnt[j] = 0;
            wave_sync();
          }
          const uint32_t d0 = l * W_DE, d1 = min(d0 + W_DE, D);
          uint32_t sn = 0; uint64_t mm = 0;
          for (uint32_t j = d0; j < d1; j++) {
            const bool sg = j == 0 || (L.dkey[j - 1] >> 32) != (L.dkey[j] >> 32);
            L.dflag[j] = sg ? 1 : 0;
            sn += sg ? 1 : 0;
          }
          const uint32_t sex = wave_exscan(sn, nseg);
          if (nseg > (uint32_t)W_BLK) st = ST_DEFER;   // segment ids index segcnt[W_BLK]
          else {
          uint32_t sidr = sex;
          for (uint32_t j = d0; j < d1; j++) {
            sidr += L.dflag[j] & 1;
            L.dflag[j] = (uint8_t)((L.dflag[j] & 3) | ((sidr - 1) << 2));
            const uint64_t v = ((uint64_t)(sidr - 1) << 32) | ((uint32_t)L.dkey[j] + L.dlen[j]);
            mm = v > mm ? v : mm;
          }
          uint64_t dmex = wave_incl_scan_max(mm); dmex = __shfl_up(dmex, 1, WAVE); if (l == 0) dmex = 0;
          uint64_t runmax = dmex; uint32_t rh = 0;
          for (uint32_t j = d0; j < d1; j++) {
            const uint32_t sidj = L.dflag[j] >> 2;
            const bool rs = (L.dflag[j] & 1) || (uint32_t)L.dkey[j] > (uint32_t)runmax;
            if (rs) { L.dflag[j] |= 2; atomicAdd(&L.segcnt[sidj], 1u); rh = j + 1; }
            const uint64_t v = ((uint64_t)sidj << 32) | ((uint32_t)L.dkey[j] + L.dlen[j]);
            runmax = v > runmax ? v : runmax;
          }
          uint32_t rhex = wave_incl_scan_max(rh); rhex = __shfl_up(rhex, 1, WAVE); if (l == 0) rhex = 0;
          uint32_t rhead = rhex;
          for (uint32_t j = d0; j < d1; j++) {
            if (L.dflag[j] & 2) rhead = j + 1;
            atomicMax(&L.drunend[rhead - 1], (uint32_t)L.dkey[j] + L.dlen[j]);
          }
          wave_sync();
          uint32_t dacc = 0;
          for (uint32_t j = d0; j < d1; j++) {
            const uint32_t cl = L.dcl[j], ck = (uint32_t)L.dkey[j];
            uint32_t sz = 0;
            if (L.dflag[j] & 1) sz += vu_len(cl) + vu_len(L.segcnt[L.dflag[j] >> 2]);
            if (L.dflag[j] & 2) sz += vu_len(ck) + vu_len(L.drunend[j] - ck);
            L.dposs[j] = (uint16_t)dacc; dacc += sz;
          }
          const uint32_t dl0 = wave_exscan(dacc, dsbytes);
          for (uint32_t j = d0; j < d1; j++) L.dposs[j] = (uint16_t)(L.dposs[j] + dl0);
          size = (uint64_t)hdr0 + sbytes + vu_len(nseg) + dsbytes;
          // the copy-out writes align16(size) bytes of the LDS buffer into the slot
          if (((size + 15) & ~15ull) > cap || size > (uint64_t)W_OUT) st = ST_DEFER;   // the workgroup kernel places it
          }
        }
      }
    }
  }
  DIAGW(5);
  if (st == ST_OK && slot + size > out_cap) st = ST_NOMEM;
  if (l == 0) {
    if (st == ST_OK) add_payload(meta, d, size);
    out_off[d] = slot; out_len[d] = st == ST_OK ? size : 0;
    status[d] = st == ST_DEFER ? ST_FALLBACK : st;
    if (st == ST_DEFER) defer_list[atomicAdd(&meta->defer_count, 1u)] = d;
    if (st == ST_FALLBACK) {
      fb_list[atomicAdd(&meta->fb_count, 1u)] = d;
      atomicAdd(&meta->fb_upds, (unsigned long long)k);
      atomicAdd(&meta->fb_bytes, (unsigned long long)nbytes);
    }
  }
  if (st != ST_OK) return;
  uint8_t* o = out + slot;
  if (mode == 1) { if (l == 0) { o[0] = 0; o[1] = 0; } return; }
  if (mode == 2) { for (uint64_t i = l; i < nbytes; i += WAVE) o[i] = arena[b0 + i]; return; }
  // ---- emit: lane-contiguous segments into the LDS output buffer
  LO8* lo = (LO8*)L.out;
  if (l == 0) { LWriter w{lo, 0}; w.vu(nC); }
  const uint32_t e0 = l * W_E, e1 = min(e0 + W_E, S);
  LWriter gw{lo, hdr0 + (e0 < S ? L.epos[e0] : sbytes)};
  for (uint32_t j = e0; j < e1; j++) {
    const uint32_t f = L.eflag[j];
    const uint64_t kj = L.key[j]; const uint32_t r = (uint32_t)kj & 0xFF;
    const uint32_t crk = (uint32_t)(kj >> 40), ck = (uint32_t)(kj >> 8);
    const uint32_t cl = L.ctab[crk];
    if (f & EF_NEWC) { gw.vu(L.blkcnt[crk]); gw.vu(cl); gw.vu(ck); }
    if (f & EF_GAP) { const uint64_t kp = L.key[j - 1]; gw.b(10); gw.vu(ck - ((uint32_t)(kp >> 8) + (uint32_t)L.ra[kp & 0xFF])); }
    if (f & EF_EMIT) {
      const uint64_t ra = L.ra[r];
      const uint32_t s0 = (uint32_t)(ra >> 48), n = (uint32_t)(ra >> 32) & 0xFFFF;
      if (f & EF_GC) { gw.b(0); gw.vu(L.rcl[j] - ck); }
      else if (!((L.rb[r] >> 13) & 4)) {  // canonical item: input bytes, info bit 0x20 dropped when an origin is set
        const uint8_t info = L.in[s0];
        gw.b((info & 0xC0) ? (uint8_t)(info & ~0x20) : info);
        gw.copy((LU8*)L.in, s0 + 1, n - 1);
      } else {
        Cur c{L.in, s0, s0 + n, 0, 0};
        SInfo si; read_struct<true>(c, si, flags);
        Out w{(uint8_t*)(lo + gw.pos), 0};
        write_struct(w, L.in, si, cl, ck, 0, false, flags);
        gw.pos += (uint32_t)w.n;
      }
    }
  }
  const uint32_t dsb = hdr0 + sbytes;
  if (l == 0) { LWriter w{lo, dsb}; w.vu(nseg); }
  const uint32_t d0 = l * W_DE, d1 = min(d0 + W_DE, D);
  LWriter dw{lo, dsb + vu_len(nseg) + (d0 < D ? L.dposs[d0] : dsbytes)};
  for (uint32_t j = d0; j < d1; j++) {
    const uint32_t cl = L.dcl[j], ck = (uint32_t)L.dkey[j];
    if (L.dflag[j] & 1) { dw.vu(cl); dw.vu(L.segcnt[L.dflag[j] >> 2]); }
    if (L.dflag[j] & 2) { dw.vu(ck); dw.vu(L.drunend[j] - ck); }
  }
  wave_sync();
  // ---- coalesced copy-out (the slot is 16-byte aligned and holds align16(size) bytes)
  const uint32_t nch = (uint32_t)((size + 15) / 16);
  for (uint32_t c = l; c < nch; c += WAVE) *(uint4*)(o + 16 * c) = *(const uint4*)(L.out + 16 * c);
  DIAGW(7);
}

// Documents deferred by the lean kernel, one wave each (persistent grid; count from device memory).
__global__ __launch_bounds__(WAVE) void k_merge_wave(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                     const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ docs,
                                                     const unsigned int* n_dev, uint32_t n_docs, uint32_t flags,
                                                     uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                                                     uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                                                     DocMeta* meta, uint32_t* defer_list, uint32_t* fb_list, uint64_t out_cap) {
  __shared__ WaveLds L;
  const uint32_t N = n_dev ? *n_dev : n_docs;
  for (uint32_t i = blockIdx.x; i < N; i += gridDim.x) {
    merge_wave_doc(L, docs ? docs[i] : i, arena, upd_off, doc_upd, flags, out, out_off, out_len, status, meta, defer_list, fb_list, out_cap);
    wave_sync();
  }
}

// The wave kernel's routing decision taken before it, one LANE per document: a [snapshot, ...log] document whose largest
// update is BIG_ROUTE_MIN bytes or more goes to the large-document tier's list (fb_list, with the scratch-sizing sums),
// every other document to `rest` (count meta->route_n), which k_merge_wave then takes.  Each list takes one atomic per
// wave.  (In k_merge_wave the decision cost a wave and three atomics on three hot counters per document: C3's 100 000
// documents spent ~2 ms there, none of them merged by it.)
__global__ __launch_bounds__(256) void k_route_big(const uint64_t* __restrict__ upd_off, const uint32_t* __restrict__ doc_upd,
                                                   const uint32_t* __restrict__ docs, const unsigned int* n_dev, uint32_t n_docs,
                                                   uint32_t flags, uint64_t* __restrict__ out_off, uint64_t* __restrict__ out_len,
                                                   int32_t* __restrict__ status, DocMeta* meta, uint32_t* __restrict__ fb_list,
                                                   uint32_t* __restrict__ rest) {
  const uint32_t N = n_dev ? *n_dev : n_docs;
  const uint32_t l = threadIdx.x % WAVE;
  for (uint32_t base = blockIdx.x * 256u; base < N; base += gridDim.x * 256u) {   // (block-uniform trip count)
    const uint32_t i = base + threadIdx.x;
    const bool in = i < N;
    const uint32_t d = in ? docs[i] : 0u;
    const uint32_t u0 = in ? doc_upd[d] : 0u, u1 = in ? doc_upd[d + 1] : 0u, k = u1 - u0;
    // as merge_wave_doc: empty and one-update documents and the forced sequential mode stay with the wave kernel
    const bool cand = in && k >= 2u && !(flags & 2u);
    // the largest update: a lane walks its document's offsets, or -- a document of more than 64 updates -- the wave
    // does, 64 offsets at a time (a lane walking 100 000 updates held its wave for milliseconds)
    const bool coop = cand && k > 64u;
    uint64_t mx = 0, prev = cand ? upd_off[u0] : 0ull;
    for (uint32_t j = 1; j <= (cand && !coop ? k : 0u); j++) {
      const uint64_t x = upd_off[u0 + j];
      mx = x - prev > mx ? x - prev : mx;
      prev = x;
    }
    for (uint64_t cm = __ballot(coop); cm; cm &= cm - 1ull) {   // (wave-uniform)
      const int src = __builtin_ctzll(cm);
      const uint32_t ua = (uint32_t)__shfl((int)u0, src), kk = (uint32_t)__shfl((int)k, src);
      uint64_t m2 = 0;
      for (uint32_t j = l; j < kk; j += WAVE) { const uint64_t n2 = upd_off[ua + j + 1] - upd_off[ua + j]; m2 = n2 > m2 ? n2 : m2; }
#pragma unroll
      for (int o = WAVE / 2; o > 0; o >>= 1) { const uint64_t t2 = __shfl_xor(m2, o, WAVE); m2 = t2 > m2 ? t2 : m2; }
      if (l == (uint32_t)src) mx = m2;
    }
    const bool big = cand && mx >= (uint64_t)BIG_ROUTE_MIN;
    const uint64_t bm = __ballot(big), rm = __ballot(in && !big);
    const uint32_t lead = (uint32_t)__builtin_ctzll(bm | (1ull << 63));
    uint32_t fb0 = 0, r0 = 0;
    if (bm) {
      const uint64_t nb = big ? upd_off[u1] - upd_off[u0] : 0ull;
      const uint64_t su = wave_sum((uint64_t)(big ? k : 0u)), sb = wave_sum(nb);
      if (l == lead) {
        fb0 = atomicAdd(&meta->fb_count, (unsigned int)__popcll(bm));
        atomicAdd(&meta->fb_upds, (unsigned long long)su);
        atomicAdd(&meta->fb_bytes, (unsigned long long)sb);
      }
      fb0 = (uint32_t)__shfl((int)fb0, (int)lead);
    }
    if (rm) {
      const uint32_t rl = (uint32_t)__builtin_ctzll(rm);
      if (l == rl) r0 = atomicAdd(&meta->route_n, (unsigned int)__popcll(rm));
      r0 = (uint32_t)__shfl((int)r0, (int)rl);
    }
    if (big) {
      fb_list[fb0 + lanes_below(bm)] = d;
      out_off[d] = merge_slot(upd_off[u0], d); out_len[d] = 0; status[d] = ST_FALLBACK;
    } else if (in) rest[r0 + lanes_below(rm)] = d;
  }
}


// ======================================================================= merge: lean fast path
// Persistent waves (ygm_merge_lean.hpp): wave w takes documents w, w + G, w + 2G, ...
// While document i is parsed, the chunk loads of document i + 1 are in flight (register
// prefetch) and the scalar header loads of documents i + 1 / i + 2 run ahead of them.
// Documents outside the lean shape are appended to `defer_list` for k_merge_wave.
// the lane id, recomputed where it is used: an address derived from threadIdx.x is loop-invariant across the
// persistent loop's documents, so the compiler hoists it out and, at the 128-VGPR cap, spills it -- and the copy
// loops then wait on a scratch reload per document
YDEV uint32_t lane_opaque() {
  uint32_t li;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(li));
  return li;
}
struct LeanHdr { uint32_t u0, k; uint64_t b0, nbytes; };

// Document headers come through VECTOR loads (lane-dependent addresses, then readlane): a
// scalar load would share lgkmcnt with the LDS traffic of the document being parsed, and
// every LDS wait would then also wait for the header's trip to memory.
YDEV uint32_t lean_du_load(const uint32_t* __restrict__ doc_upd, uint32_t d, uint32_t n_docs) {
  const uint32_t l = threadIdx.x;
  return d < n_docs ? doc_upd[d + (l & 1u)] : 0u;          // lanes 0 / 1: doc_upd[d], doc_upd[d + 1]
}
// document bytes [b0, b1): lanes 0 / 1 load b0 / b1 -- from the update-offset table, or (LENS) from the per-document
// offsets of the compact input form (ygm_merge_v1_device_lens: u64 per document, u16 length per update)
template <int LENS>
YDEV uint64_t lean_bo_load(const uint64_t* __restrict__ upd_off, const uint64_t* __restrict__ doc_off, uint32_t du, uint32_t d,
                           uint32_t n_docs) {
  if (LENS) return d < n_docs ? doc_off[d + (threadIdx.x & 1u)] : 0ull;
  const uint32_t u0 = rdlane(du, 0), u1 = rdlane(du, 1);
  return d < n_docs ? upd_off[(threadIdx.x & 1u) ? u1 : u0] : 0ull;
}
YDEV LeanHdr lean_hdr_of(uint32_t du, uint64_t bo) {
  LeanHdr h;
  h.u0 = rdlane(du, 0); h.k = rdlane(du, 1) - h.u0;
  const uint64_t b0 = ((uint64_t)rdlane((uint32_t)(bo >> 32), 0) << 32) | rdlane((uint32_t)bo, 0);
  const uint64_t b1 = ((uint64_t)rdlane((uint32_t)(bo >> 32), 1) << 32) | rdlane((uint32_t)bo, 1);
  h.b0 = b0; h.nbytes = b1 - b0;
  return h;
}
template <int WIDE>
YDEV bool lean_stageable(const LeanHdr& h) {
  return h.k >= 2 && h.k < (uint32_t)(WAVE * LN_ROWS) && (h.b0 & 15u) + h.nbytes <= (uint64_t)LnCfg<WIDE>::IN;
}
// issues the loads of one document: staged chunks and the per-row update offsets.  Every
// load is unconditional (clamped addresses) so the prefetch registers are dead between the
// staging of one document and the prefetch of the next (no loop-carried live ranges).
template <int WIDE, int LENS = 0>
YDEV void lean_prefetch(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off, const uint16_t* __restrict__ upd_len,
                        const LeanHdr& h, bool go, u32x4 (&v)[(LnCfg<WIDE>::IN + 16 * WAVE - 1) / (16 * WAVE)], uint32_t (&rx)[LN_ROWS],
                        uint32_t (&ry)[LN_ROWS]) {
  const uint32_t l = threadIdx.x;
  const uint64_t a0 = go ? (h.b0 & ~15ull) : 0ull;
  const uint32_t last = go ? (uint32_t)(((h.b0 & 15u) + h.nbytes + 15) / 16) - 1u : 0u;
#pragma unroll
  for (int j = 0; j < (LnCfg<WIDE>::IN + 16 * WAVE - 1) / (16 * WAVE); j++) {
    const uint32_t c = l + WAVE * j;
    v[j] = *(const u32x4*)(arena + a0 + 16ull * (c < last ? c : last));
  }
  // low dwords only (offsets inside one document differ by < 2^32; whole-register loads keep
  // the allocator from reusing a dead high half while the load is in flight -- a forced wait)
  const uint32_t kk = go ? h.k : 0u;
  if (LENS) {   // the rows' update lengths (2 bytes each); offsets by a scan at staging
#pragma unroll
    for (int q = 0; q < LN_ROWS; q++) {
      const uint32_t i = l + WAVE * q;
      rx[q] = upd_len[h.u0 + (i < kk ? i : 0u)];
    }
    return;
  }
  const uint32_t* off32 = (const uint32_t*)upd_off;
#pragma unroll
  for (int q = 0; q < LN_ROWS; q++) {
    const uint32_t i = l + WAVE * q;
    const uint32_t ix = h.u0 + (i < kk ? i : 0u);
    rx[q] = off32[2ull * ix]; ry[q] = off32[2ull * ix + 2];
  }
}

// WIDE = 0: the narrow kernel over every document of the batch (wave w: documents w, w + G, ...), which zeroes
// the next launch's counter slot.  WIDE = 1: the wide kernel (LnCfg<1>) over the narrow kernel's deferred
// list (wave w: entries w, w + G, ... of `list`), deferring in turn to its own list (meta->wide_defer).
template <int WIDE, int LENS = 0>
#ifndef YGM_LN_OCC
#define YGM_LN_OCC 4   // waves per SIMD the narrow kernel's registers are cut for (its LDS allows 160 KB / (in + out) per CU)
#endif
__global__ __launch_bounds__(WAVE, WIDE ? 3 : YGM_LN_OCC) void k_merge_lean(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                     const uint32_t* __restrict__ doc_upd, uint32_t n_docs, uint32_t flags,
                                                     uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                                                     uint64_t* __restrict__ out_len, int32_t* __restrict__ status, DocMeta* meta,
                                                     DocMeta* __restrict__ meta_next, uint32_t* __restrict__ defer_list, uint64_t out_cap,
                                                     const uint32_t* __restrict__ list, uint32_t n_list,
                                                     const uint64_t* __restrict__ doc_off, const uint16_t* __restrict__ upd_len) {
  typedef LnCfg<WIDE> C;
  __shared__ LeanLdsT<WIDE> LS;
  if (meta_next && blockIdx.x == 0) {   // the next launch's counter slot (nothing reads it during this launch)
    static_assert(sizeof(DocMeta) % 16 == 0, "DocMeta is zeroed in 16-byte pieces");
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (uint32_t i = threadIdx.x; i < sizeof(DocMeta) / 16; i += WAVE) ((u32x4*)meta_next)[i] = z;
  }
  LB8* lin = (LB8*)LS.in;
  LB8* lout = (LB8*)LS.out;
  const uint32_t l = threadIdx.x;
  const uint32_t G = gridDim.x;
  const bool force_seq = (flags & 2u) != 0;
  // the wave's j-th document: blockIdx.x + j G (narrow), or list entry blockIdx.x + j G (wide; n_docs past the list).
  // Wide: lane l of lst0 / lst1 holds the entry of iteration 64 b + l / 64 (b + 1) + l (b = the current run)
  const uint32_t n_it = WIDE ? n_list : n_docs;
  auto list_at = [&](uint32_t j) -> uint32_t {   // (list == nullptr: every document of the batch, the wide route)
    const uint64_t i = (uint64_t)blockIdx.x + (uint64_t)j * G;
    return i < n_it ? (list ? list[i] : (uint32_t)i) : n_docs;
  };
  uint32_t lst0 = 0, lst1 = 0;
  if (WIDE) { lst0 = list_at(l); lst1 = list_at(WAVE + l); }
  uint32_t it = 0;
  auto docof = [&](uint32_t j) -> uint32_t {   // (j within the current run or the next)
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)rdlane((j >> 6) != (it >> 6) ? lst1 : lst0, j & 63u));
  };
  // the document k places after the current one (narrow: d is the induction variable)
#define LN_AHEAD(k) (WIDE ? docof(it + (k)) : d + (k) * G)
  uint32_t d = WIDE ? (n_it > blockIdx.x ? docof(0) : n_docs) : blockIdx.x;
  (void)n_it;
  uint32_t du = lean_du_load(doc_upd, d, n_docs);
  LeanHdr hn = lean_hdr_of(du, lean_bo_load<LENS>(upd_off, doc_off, du, d, n_docs));
  du = lean_du_load(doc_upd, LN_AHEAD(1), n_docs);                  // header pipeline: doc_upd one document ahead
  u32x4 v[(C::IN + 16 * WAVE - 1) / (16 * WAVE)];
  uint32_t rx[LN_ROWS], ry[LN_ROWS];
#pragma unroll
  for (int q = 0; q < LN_ROWS; q++) { rx[q] = 0; ry[q] = 0; }
  bool gn = !force_seq && lean_stageable<WIDE>(hn);
  lean_prefetch<WIDE, LENS>(arena, upd_off, upd_len, hn, gn, v, rx, ry);
  uint64_t payload = 0;   // this wave's output bytes: one atomic per wave, not per document
  // deferred documents: bit j of dmask = the j-th document of the current run of 64 iterations (document
  // dch + j * G), appended to defer_list with ONE atomic per run -- one atomic per document on the single
  // counter serialises a batch the lean kernel mostly defers (10 000 documents: ~80 us)
  uint64_t dmask = 0;
  uint32_t dit = 0, dch = d;
  auto flush_defer = [&]() {
    if (!dmask) return;
    uint32_t base = 0;
    if (l == 0) base = atomicAdd(WIDE ? &meta->wide_defer : &meta->lean_defer, (uint32_t)__popcll(dmask));
    base = __shfl(base, 0, WAVE);
    if ((dmask >> l) & 1ull) defer_list[base + (uint32_t)__popcll(dmask & ((1ull << l) - 1ull))] = WIDE ? lst0 : dch + l * G;
    dmask = 0;
  };
  for (; WIDE ? (uint64_t)blockIdx.x + (uint64_t)it * G < n_it : d < n_docs; it++) {
    DIAGL_T0
    if (dit == 64) {
      flush_defer(); dit = 0; dch = d;
      if (WIDE) { lst0 = lst1; lst1 = list_at(it + WAVE + l); }   // the run's entries move down; the next run's are loaded
    }
    const LeanHdr h = hn;
    bool go = gn;
    const uint32_t k = h.k;
    const uint64_t b0 = h.b0, nbytes = h.nbytes;
    const uint64_t slot = merge_slot(b0, d), cap = merge_slot_cap(nbytes);
    const uint32_t shift = (uint32_t)(b0 & 15u);
    // ---- stage the prefetched document into LDS
    uint32_t us[LN_ROWS], un[LN_ROWS];
    if (go) {
      const uint32_t nch = (uint32_t)((shift + nbytes + 15) / 16);
#pragma unroll
      for (int j = 0; j < (C::IN + 16 * WAVE - 1) / (16 * WAVE); j++) {
        const uint32_t c = l + WAVE * j;
        if (c < nch) *(LB128*)(lin + 16 * c) = v[j];
      }
      if (LENS) {   // offsets: an exclusive scan of the lengths over rows (update l + 64 q in lane l of row q)
        uint32_t carry = shift;
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) {
          un[q] = l + WAVE * q < k ? rx[q] : 0u;
          const uint32_t inc = dpp_incl_add(un[q]);
          us[q] = carry + inc - un[q];
          carry += lane63(inc);
        }
        if (carry - shift != (uint32_t)nbytes) go = false;   // lengths that do not add up: deferred (k_build_off clamps)
      } else {
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) { us[q] = shift + (rx[q] - (uint32_t)b0); un[q] = ry[q] - rx[q]; }
      }
      if (!WIDE) {   // an update past the narrow window: the wide kernel's document -- defer it without parsing
        bool lng = false;
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) lng |= l + WAVE * q < k && un[q] > (uint32_t)LN_UMAX;
        if (__ballot(lng)) go = false;
      }
    }
    // every prefetch load has landed on every path (free after the staging): without this the waitcnt
    // pass, path-insensitive, sees them pending in the parse and makes it wait -- counters being in
    // order -- for the next header's loads issued below
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    wave_sync();
    DIAGL(0);
#if defined(YGM_LEAN_STOP) && YGM_LEAN_STOP == 1   // timing experiment: stage only
    { hn = lean_hdr_of(du, lean_bo_load<LENS>(upd_off, doc_off, du, LN_AHEAD(1), n_docs)); du = lean_du_load(doc_upd, LN_AHEAD(2), n_docs);
      gn = !force_seq && lean_stageable<WIDE>(hn); lean_prefetch<WIDE, LENS>(arena, upd_off, upd_len, hn, gn, v, rx, ry); wave_sync(); dit++; d = LN_AHEAD(1); continue; }
#endif
    // ---- header of the next document (its prefetch is issued after the parse) and doc_upd of the one after
    const uint64_t bo_next = lean_bo_load<LENS>(upd_off, doc_off, du, LN_AHEAD(1), n_docs);
    const uint32_t du_next = lean_du_load(doc_upd, LN_AHEAD(2), n_docs);
    // single: mergeUpdates([]) = 0000; a single input is returned as is (Y@39011).  It shares the
    // prefetch below with the parse path (a prefetch of its own, in its own branch, gets hoisted
    // above the branch and the parse then waits on those loads)
    const bool single = k < 2 && !force_seq;
    bool defer = !go && !single;
    uint32_t size = 0;
    if (single) {
      size = k == 0 ? 2u : (uint32_t)nbytes;
      if (k == 1 && nbytes > 0xFFFFFFFFull) size = 0;
      uint8_t* o = out + slot;
      // compact input form: a single update whose length is not the document's bytes (include/ygm.h: an error)
      const bool badlen = upd_len != nullptr && k == 1 && (uint64_t)upd_len[h.u0] != nbytes;
      if (badlen) { size = 0; if (l == 0) { out_off[d] = slot; out_len[d] = 0; status[d] = ST_MALFORMED; } }
      else if (slot + (k == 0 ? 2 : nbytes) > out_cap) { size = 0; if (l == 0) { out_off[d] = slot; out_len[d] = 0; status[d] = ST_NOMEM; } }
      else {
        if (k == 0) { if (l == 0) { o[0] = 0; o[1] = 0; } }
        else for (uint64_t c = lane_opaque(); c * 16 < nbytes; c += WAVE) {   // unaligned 16-byte loads (arena tail padding >= 16), aligned stores
          uint4 x; __builtin_memcpy(&x, arena + b0 + 16 * c, 16);
          *(uint4*)(o + 16 * c) = x;
        }
        if (l == 0) { out_off[d] = slot; out_len[d] = k == 0 ? 2 : nbytes; status[d] = ST_OK; }
        payload += k == 0 ? 2 : nbytes;
      }
      // drain the copy's loads here: left pending into the join with the parse path, the waitcnt pass
      // makes the parse wait for them -- and, counters being in order, for the next header's loads
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    }
    // ---- parse, lane per update
    LRec rec[LN_ROWS];
    bool hs[LN_ROWS], hasd[LN_ROWS];   // row holds an update with structs / with a non-empty delete set
    bool bad = false;
#pragma unroll
    for (int q = 0; q < LN_ROWS; q++) { hs[q] = false; hasd[q] = false; }
    if (go) {
#pragma unroll
      for (int q = 0; q < LN_ROWS; q++) {
        const bool valid = l + WAVE * q < k;
        if (valid) { rec[q] = lean_parse<WIDE ? LNW_UMAX : LN_UMAX>(lin, us[q], un[q]); bad |= !rec[q].ok; }
        else { rec[q].ok = true; rec[q].client = 0; rec[q].clock = 0; rec[q].clen = 0; rec[q].span = 0; }
        hs[q] = valid && (rec[q].span & 0xFF00u) != 0u;
        hasd[q] = valid && rec[q].ok && lin[lean_ds_pos(us[q], rec[q].span)] != 0;
      }
    }
    DIAGL(1);
    // ---- prefetch the next document while this one is scanned and emitted (kept below the parse:
    //      hoisted above it, the parse waits on the prefetch's vmcnt)
#ifdef YGM_LEAN_SB
    __builtin_amdgcn_sched_barrier(0);
#endif
    hn = lean_hdr_of(du, bo_next); du = du_next;
    gn = !force_seq && lean_stageable<WIDE>(hn);
    lean_prefetch<WIDE, LENS>(arena, upd_off, upd_len, hn, gn, v, rx, ry);
    defer = defer || __ballot(bad) != 0;
    if (single) { wave_sync(); dit++; d = LN_AHEAD(1); continue; }   // (dit: bit j of dmask is the run's j-th document)
#if defined(YGM_LEAN_STOP) && YGM_LEAN_STOP == 2   // timing experiment: stage + parse
    if (l == 0) status[d] = (int)bad; wave_sync(); dit++; d = LN_AHEAD(1); continue;
#endif
    if (!defer) {
      // ---- clients, discovered in descending order (wave max over the unassigned records): a
      //      record's block is its client's rank; lane c of `ctl` holds block c's client
      uint32_t blk[LN_ROWS];
#pragma unroll
      for (int q = 0; q < LN_ROWS; q++) blk[q] = hs[q] ? 0xFFu : 0xFEu;
      uint32_t ctl = 0, nC = 0;
      for (int it = 0; it <= LN_CMAX; it++) {
        uint32_t mx = 0; bool any = false;
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) { const bool un_ = blk[q] == 0xFFu; any |= un_; mx = max(mx, un_ ? rec[q].client : 0u); }
        if (__ballot(any) == 0) break;
        if (nC == (uint32_t)LN_CMAX) { defer = true; break; }
        const uint32_t cand = lane63(dpp_incl_max(mx));
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) if (blk[q] == 0xFFu && rec[q].client == cand) blk[q] = nC;
        ctl = l == nC ? cand : ctl;
        nC++;
      }
      if (!defer) {
        // ---- record index inside its block: per-row DPP scans of packed 8-bit per-block counts (k <= 255)
        uint32_t cA = 0, cB = 0;
        uint32_t idx[LN_ROWS];
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) {
          const uint32_t b = hs[q] ? blk[q] : 0u;
          const uint32_t sh = 8u * (b & 3u);
          const uint32_t pa = (hs[q] && b < 4u) ? 1u << sh : 0u;
          const uint32_t ia = dpp_incl_add(pa);
          uint32_t w = cA + ia - pa;
          cA += lane63(ia);
          if (nC > 4u) {
            const uint32_t pb = (hs[q] && b >= 4u) ? 1u << sh : 0u;
            const uint32_t ib = dpp_incl_add(pb);
            w = b < 4u ? w : cB + ib - pb;
            cB += lane63(ib);
          }
          idx[q] = (w >> sh) & 0xFFu;
        }
        // exclusive per-block record bases, packed 8-bit (blocks 0-3 / 4-7): the prefix sum of the
        // packed counts by byte (x * 0x01010100 adds every lower byte into the higher ones)
        const uint32_t RB0 = cA * 0x01010100u;
        const uint32_t tot0 = (RB0 >> 24) + (cA >> 24);
        const uint32_t RB1 = cB * 0x01010100u + tot0 * 0x01010101u;
        const uint32_t nrec = (RB1 >> 24) + (cB >> 24);
        // ---- records scattered to their sorted slot (block, log order): clock, end, packed source
        //      (staged position << 16 | block << 13 | structs << 5 | struct bytes)
        LB32* Sck = (LB32*)lout;
        LB32* Sen = Sck + WAVE * LN_ROWS;
        LB32* Ssp = Sen + WAVE * LN_ROWS;
        LB32* Sbs = Ssp + WAVE * LN_ROWS;   // per block: packed (structs, bytes) before its first record; first clock
        LB32* Sfc = Sbs + LN_CMAX;
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) {
          if (hs[q]) {
            const uint32_t b = blk[q];
            const uint32_t j = idx[q] + ((b < 4u ? RB0 : RB1) >> (8u * (b & 3u)) & 0xFFu);
            Sck[j] = rec[q].clock; Sen[j] = rec[q].clock + rec[q].clen;
            Ssp[j] = (rec[q].span & 0xFFFF0000u) | (b << 13) | (((rec[q].span >> 8) & 0x7Fu) << 6) | (rec[q].span & 0x3Fu);
          }
        }
        wave_sync();
        // ---- sorted domain: contiguity (rule R-M without gaps / overlaps: a record's clock is the end
        //      of the previous record of its block) and the packed (structs, bytes) prefix
        uint32_t osp[LN_ROWS], oex[LN_ROWS];
        uint32_t carry = 0;
#pragma unroll
        for (int r = 0; r < LN_ROWS; r++) {
          const uint32_t j = l + WAVE * r;
          const bool v = j < nrec;
          const uint32_t sp = v ? Ssp[j] : 0u, ck = v ? Sck[j] : 0u;
          const uint32_t spp = (v && j > 0u) ? Ssp[j - 1u] : 0u, ep = (v && j > 0u) ? Sen[j - 1u] : 0u;
          const bool first = v && (j == 0u || ((spp ^ sp) & 0xE000u) != 0u);   // first record of its block
          bad |= v && !first && ck != ep;
          const uint32_t f = v ? (((sp >> 6) & 0x7Fu) << 16) | (sp & 0x3Fu) : 0u;
          const uint32_t inc = carry + dpp_incl_add(f);
          const uint32_t ex = inc - f;
          carry = lane63(inc);
          if (first) { Sbs[(sp >> 13) & 7u] = ex; Sfc[(sp >> 13) & 7u] = ck; }
          osp[r] = sp; oex[r] = ex;
        }
        wave_sync();
        // ---- block headers, lane c = block c: structs, client, first clock; header offsets by a scan
        uint32_t hcnt = 0, hfc = 0, hbs = 0, hlen = 0;
        if (l < nC) {
          hbs = Sbs[l]; hfc = Sfc[l];
          const uint32_t nxt = l + 1u < nC ? Sbs[l + 1u] : carry;
          hcnt = (nxt >> 16) - (hbs >> 16);
          hlen = vu_len(hcnt) + vu_len(ctl) + vu_len(hfc);
        }
        const uint32_t hinc = dpp_incl_add(hlen);          // header bytes of blocks <= c (< 128 with <= 8 blocks)
        const uint32_t hdr_all = lane63(hinc);
        uint32_t HC0 = 0, HC1 = 0;                         // vu_len(nC) + hinc of each block, packed 8-bit
#pragma unroll
        for (int c = 0; c < LN_CMAX; c++) {
          const uint32_t hc = rdlane(hinc, (uint32_t)c) + vu_len(nC);
          if (c < 4) HC0 |= (hc & 0xFFu) << (8 * c); else HC1 |= (hc & 0xFFu) << (8 * (c - 4));
        }
        const uint32_t hpos = vu_len(nC) + hinc - hlen + (hbs & 0xFFFFu);   // lane c: block c's header position
        wave_sync();
        // ---- delete sets: union of every update's ranges (scratch: the sorted records are consumed)
        LDsUnion dsu; dsu.bytes = 1u; dsu.bad = false; dsu.nsegs = 0;
        bool anyds = false;
#pragma unroll
        for (int q = 0; q < LN_ROWS; q++) anyds |= hasd[q];
        DIAG_PUT(6, DIAG_NOW());
        if (__ballot(anyds) != 0) {
          uint32_t dpos[LN_ROWS], uend[LN_ROWS];
#pragma unroll
          for (int q = 0; q < LN_ROWS; q++) { dpos[q] = lean_ds_pos(us[q], rec[q].span); uend[q] = us[q] + un[q]; }
          dsu = lean_ds_union(lin, (LB32*)lout, dpos, uend, hasd, flags);
          bad |= dsu.bad;
          wave_sync();
        }
        DIAG_PUT(7, DIAG_NOW());
        // the output buffer is assembled by OR: zero it
        {
          const u32x4 z = {0u, 0u, 0u, 0u};
          constexpr int NZ = (C::OUT + 80) / 16;   // 16-byte pieces of the output buffer
#pragma unroll
          for (int j = 0; j < NZ / WAVE; j++) *(LB128*)(lout + 16 * (l + WAVE * j)) = z;
          if (l < (uint32_t)(NZ % WAVE)) *(LB128*)(lout + 16 * (l + WAVE * (NZ / WAVE))) = z;
        }
        DIAGL(2);
        defer = __ballot(bad) != 0;
#if defined(YGM_LEAN_STOP) && YGM_LEAN_STOP == 3   // timing experiment: stage + parse + scan
        if (l == 0) status[d] = (int)bad + (int)(oex[0] & 1) + (int)(oex[1] & 1) + (int)(oex[2] & 1) + (int)(oex[3] & 1); wave_sync(); dit++; d = LN_AHEAD(1); continue;
#endif
        if (!defer) {
          const uint32_t at = vu_len(nC) + hdr_all;   // + the struct bytes: the delete set's position
          size = at + (carry & 0xFFFFu) + dsu.bytes;   // headers + struct bytes + the delete set
          if (size > (uint32_t)C::OUT || ((size + 15u) & ~15u) > cap || slot + size > out_cap) defer = true;
          else {
            // ---- emit into the LDS output buffer: structs (funnel copies), block headers, document header, delete set
#pragma unroll
            for (int r = 0; r < LN_ROWS; r++) {
              const uint32_t j = l + WAVE * r;
              const uint32_t b = (osp[r] >> 13) & 7u;
              const uint32_t t = (oex[r] & 0xFFFFu) + ((b < 4u ? HC0 : HC1) >> (8u * (b & 3u)) & 0xFFu);
              lean_copy<WIDE>(lout, lin, j < nrec, t, osp[r] >> 16, osp[r] & 0x3Fu);
            }
            if (l < nC) {
              uint32_t t = lds_vu(lout, hpos, hcnt);
              t = lds_vu(lout, t, ctl);
              lds_vu(lout, t, hfc);
            }
            if (l == 0) lds_vu(lout, 0, nC);
            if (dsu.bytes > 1u) lean_ds_emit(lout, at + (carry & 0xFFFFu), dsu);   // (an empty delete set is the zero byte already there)
            wave_sync();
            DIAGL(3);
            uint8_t* o = out + slot;
            const uint32_t nco = (size + 15u) / 16u;
            for (uint32_t c = lane_opaque(); c < nco; c += WAVE) *(u32x4*)(o + 16 * c) = *(const LB128*)(lout + 16 * c);
          }
        }
      }
    }
    if (!defer) payload += size;
    if (l == 0) {
      if (defer) status[d] = ST_FALLBACK;
      else { out_off[d] = slot; out_len[d] = size; status[d] = ST_OK; }
    }
    if (__builtin_amdgcn_readfirstlane((int)defer)) dmask |= 1ull << dit;   // (wave-uniform: scalar registers)
    dit++;
    DIAGL(4);
    wave_sync();   // the next document's staging overwrites lin / lout
    d = LN_AHEAD(1);
  }
  flush_defer();
  if (l == 0 && payload) add_payload(meta, blockIdx.x, payload);
#undef LN_AHEAD
}

// ======================================================================= merge: large documents
// One wave per document the workgroup tier sent on (ygm_merge_big.hpp); documents outside its class
// go on to the sequential kernel through fb2_list.
template <class T>
YDEV void big_bitonic(T* a, uint32_t n) {   // ascending by key; n <= 1024 (entries [n, pow2) padded)
  uint32_t P = 1;
  while (P < n) P <<= 1;
  const uint32_t l = threadIdx.x % WAVE;   // (one wave sorts: the lane, whichever wave of the workgroup it is)
  for (uint32_t i = n + l; i < P; i += WAVE) a[i].key = ~0ull;
  wave_sync();
  for (uint32_t k = 2; k <= P; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = l; i < P; i += WAVE) {
        const uint32_t x = i ^ j;
        if (x > i) {
          const T A = a[i], B = a[x];
          if ((A.key > B.key) == ((i & k) == 0)) { a[i] = B; a[x] = A; }
        }
      }
      wave_sync();
    }
}
// a workgroup sort of n <= NT * k entries by key: every entry's rank (the keys before it, ties by index: a stable
// order) from a broadcast scan of the keys, then a scatter through tmp (LDS) and the copy back
template <class T, uint32_t NT>
YDEV void big_rank_sort(T* a, uint32_t n, T* tmp, uint32_t t0) {
  for (uint32_t i = t0; i < n; i += NT) {
    const uint64_t ki = a[i].key;
    uint32_t r = 0;
#pragma unroll 4
    for (uint32_t j = 0; j < n; j++) { const uint64_t kj = a[j].key; r += (kj < ki || (kj == ki && j < i)) ? 1u : 0u; }
    tmp[r] = a[i];
  }
  __syncthreads();
  for (uint32_t i = t0; i < n; i += NT) a[i] = tmp[i];
  __syncthreads();
}
YDEV void big_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {   // the wave copies n bytes, 16 per lane-step
  for (uint64_t c = 16ull * (threadIdx.x % WAVE); c < n; c += 16ull * WAVE) {
    if (c + 16 <= n) { uint4 v; __builtin_memcpy(&v, src + c, 16); __builtin_memcpy(dst + c, &v, 16); }
    else for (uint64_t q = c; q < n; q++) dst[q] = src[q];
  }
}
// A list of byte copies (LDS) run by the wave at once: every lane takes 16-byte chunks of the whole list (the entry
// by binary search over the chunk prefix), four chunks in flight per lane, so the loads of many short copies overlap
// instead of each copy waiting for its own.  Sources may be read up to 15 bytes past their end (the arena's and
// U0's tail padding); destinations are written exactly.
struct BigCp { uint64_t src; uint32_t dst, n; };
// the chunks [c, tot) of entries cl[0, m) (pre: their inclusive chunk prefix) taken by one wave, stepping over the
// chunks of `stride` waves: four 16-byte chunks in flight per lane
// pbits (nullptr: none): U0 positions [pu0, pu0 + pn0) whose byte loses bit 0x20 (big_validate) -- applied to the chunks
// read from U0 (one 64-bit bitmap load per such chunk)
YDEV uint32_t big_patch_bytes(uint32_t nib) {   // 0x20 in byte i for bit i of nib
  return ((nib & 1u) ? 0x20u : 0u) | ((nib & 2u) ? 0x2000u : 0u) | ((nib & 4u) ? 0x200000u : 0u) | ((nib & 8u) ? 0x20000000u : 0u);
}
YDEV void big_copy_chunks(uint8_t* o, const BigCp* cl, uint32_t m, const uint32_t* pre, uint32_t tot, uint32_t c, uint32_t stride,
                          const uint32_t* pbits = nullptr, const uint8_t* pu0 = nullptr, uint32_t pn0 = 0) {
  const uint32_t l = threadIdx.x % WAVE;
  for (uint32_t c0 = c; c0 < tot; c0 += stride) {
    uint4 v[4]; uint8_t* d[4]; uint32_t k[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t c = c0 + (uint32_t)u * WAVE + l;
      k[u] = 0; d[u] = nullptr;
      if (c < tot) {
        uint32_t lo = 0, hi = m - 1;                  // first entry whose inclusive prefix exceeds c
        while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (pre[md] > c) hi = md; else lo = md + 1u; }
        const BigCp E = cl[lo];
        const uint32_t off = 16u * (c - (lo ? pre[lo - 1] : 0u));
        k[u] = E.n - off < 16u ? E.n - off : 16u;
        d[u] = o + E.dst + off;
        __builtin_memcpy(&v[u], (const uint8_t*)(uintptr_t)E.src + off, 16);
        if (pbits) {   // (wave-uniform)
          const uint64_t sa = E.src + off, ua = (uint64_t)(uintptr_t)pu0;
          if (sa >= ua && sa < ua + pn0) {
            const uint32_t p = (uint32_t)(sa - ua);
            const uint64_t bw = ((uint64_t)pbits[(p >> 5) + 1u] << 32) | pbits[p >> 5];
            const uint32_t pm = (uint32_t)(bw >> (p & 31u)) & 0xFFFFu;
            if (pm) {
              v[u].x &= ~big_patch_bytes(pm & 15u); v[u].y &= ~big_patch_bytes((pm >> 4) & 15u);
              v[u].z &= ~big_patch_bytes((pm >> 8) & 15u); v[u].w &= ~big_patch_bytes(pm >> 12);
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (k[u] == 16u) __builtin_memcpy(d[u], &v[u], 16);
      else if (k[u]) {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        for (uint32_t q = 0; q < k[u]; q++) d[u][q] = (uint8_t)(w[q >> 2] >> (8u * (q & 3u)));
      }
    }
  }
}
YDEV uint32_t big_copy_pre(const BigCp* cl, uint32_t m, uint32_t* pre) {   // the wave: chunk prefix of cl[0, m <= 64)
  const uint32_t l = threadIdx.x % WAVE;
  const uint32_t ch = l < m ? (cl[l].n + 15u) / 16u : 0u;
  const uint32_t inc = dpp_incl_add(ch);
  pre[l] = inc;
  return lane63(inc);
}
YDEV void big_copy_list(uint8_t* o, const BigCp* cl, uint32_t nc, uint32_t* pre, const uint32_t* pbits = nullptr,
                        const uint8_t* pu0 = nullptr, uint32_t pn0 = 0) {   // pre: 64 words of LDS
  for (uint32_t g = 0; g < nc; g += WAVE) {
    const uint32_t m = nc - g < (uint32_t)WAVE ? nc - g : (uint32_t)WAVE;
    const uint32_t tot = big_copy_pre(cl + g, m, pre);
    wave_sync();
    big_copy_chunks(o, cl + g, m, pre, tot, 0u, 4u * WAVE, pbits, pu0, pn0);
    wave_sync();
  }
}
// k_merge_big's command to its helper waves (cmd 0 done, 1 tile's jump tables, 2 validate the walk's struct records, 3
// clock ranges, 4 delete-set canonical check, 5 a run of the emit's copy list, 6 the log's sort)
struct BigCmd { uint32_t cmd, at, mis, tn, tb, n0; uint64_t vs, ns, sbase; const uint8_t* u0p; const uint32_t* aux; };
// output sink: pass 0 counts, pass 1 stores (lane 0 writes literals; copies go to an LDS list run by the wave when
// it fills and at the end of the pass -- consecutive ones merged)
struct BigOut {
  uint8_t* o; uint64_t n; bool w;
  BigCp* cl; uint32_t nc, cap, *pre;
  uint64_t ls, ld, le;                                  // the last entry: source, destination, destination end
  BigCmd* cmd = nullptr; uint32_t nw = 1;               // k_merge_big: the workgroup's waves run the list (cmd 5)
  const uint32_t* pbits = nullptr; const uint8_t* pu0 = nullptr; uint32_t pn0 = 0;   // U0's bytes to patch (big_copy_chunks)
  YDEV void b(uint32_t v) { if (w && threadIdx.x % WAVE == 0) o[n] = (uint8_t)v; n++; }   // (lane 0 of the writing wave)
  YDEV void vu(uint64_t v) { while (v > 127) { b(0x80u | (uint32_t)(v & 127)); v >>= 7; } b((uint32_t)v); }
  YDEV void flush() {
    if (!nc) return;
    wave_sync();
    if (!cmd) big_copy_list(o, cl, nc, pre, pbits, pu0, pn0);
    else   // 64 entries per command: wave 0 publishes their chunk prefix, every wave takes every nw-th run of chunks
      for (uint32_t g = 0; g < nc; g += WAVE) {
        const uint32_t m = nc - g < (uint32_t)WAVE ? nc - g : (uint32_t)WAVE;
        const uint32_t tot = big_copy_pre(cl + g, m, pre);
        if (threadIdx.x % WAVE == 0) {
          cmd->cmd = 5; cmd->vs = (uint64_t)(uintptr_t)(cl + g); cmd->ns = m; cmd->u0p = o; cmd->tb = tot;
          cmd->aux = pbits; cmd->sbase = (uint64_t)(uintptr_t)pu0; cmd->n0 = pn0;
        }
        __syncthreads();
        big_copy_chunks(o, cl + g, m, pre, tot, 0u, nw * 4u * WAVE, pbits, pu0, pn0);
        __syncthreads();
      }
    nc = 0;
  }
  YDEV void add(uint64_t src, uint64_t dst, uint64_t len) {
    for (uint64_t a = 0; a < len; a += (1ull << 29)) add1(src + a, dst + a, len - a < (1ull << 29) ? len - a : (1ull << 29));
  }
  YDEV void add1(uint64_t src, uint64_t dst, uint64_t len) {   // len < 2^30
    if (nc && le == dst && ls + (le - ld) == src && le - ld + len < (1ull << 30)) {   // continues the last entry
      if (threadIdx.x % WAVE == 0) cl[nc - 1].n = (uint32_t)(le - ld + len);
    } else {
      if (nc == cap) flush();
      if (threadIdx.x % WAVE == 0) { BigCp E; E.src = src; E.dst = (uint32_t)dst; E.n = (uint32_t)len; cl[nc] = E; }
      nc++; ls = src; ld = dst;
    }
    le = dst + len;
  }
  YDEV void copy(const uint8_t* s, uint64_t len) {
    if (w) add((uint64_t)(uintptr_t)s, n, len);
    n += len;
  }
};
// U0's delete set, decoded once by the wave into u32 values (big_ds_decode), then read as a stream of
// ranges by every lane redundantly (same values, same state): 64 values per register, lane j holding
// value b + j, taken by readlane with a uniform index; the next 64 are in flight while these are read.
struct VStream {
  const uint32_t* V; uint32_t n, i, b, cur, nxt; bool err;
  YDEV uint32_t fetch(uint32_t at) const { const uint32_t j = at + threadIdx.x % WAVE; return j < n ? V[j] : 0u; }
  YDEV void init(const uint32_t* v, uint32_t nv) { V = v; n = nv; i = 0; b = 0; err = false; cur = fetch(0); nxt = fetch(WAVE); }
  YDEV uint32_t next() {
    if (i >= n) { err = true; return 0u; }
    if (i - b >= (uint32_t)WAVE) { b += WAVE; cur = nxt; nxt = fetch(b + WAVE); }
    return (uint32_t)__builtin_amdgcn_readlane((int)cur, (int)(i++ - b));
  }
};
struct BigDs {
  VStream s; uint64_t cl_left, r_left, client; bool has; uint64_t key, len;
  YDEV void next() {
    has = false;
    while (r_left == 0 && cl_left > 0 && !s.err) { client = s.next(); r_left = s.next(); cl_left--; }
    if (r_left == 0 || s.err) return;
    const uint64_t ck = s.next(); len = s.next(); r_left--;
    key = ((uint64_t)(0xFFFFFFFFu - (uint32_t)client) << 32) | ck;
    has = !s.err;
  }
};
// The delete set [ds0, n0) of U0 as u32 values V[0, nv): the wave takes 1 KiB per round, a lane per
// 16-byte chunk; varuint terminators (top bit clear) by mask, value indices by a wave prefix count, each
// value decoded by the lane holding its terminator from the 8 bytes ending there.  A trailing
// unterminated varuint is not a value (the stream runs out if it is needed).  false: a varuint of more
// than 5 bytes or above 2^32 - 1, or more values than `cap` (the general path takes the document).
YDEV bool big_ds_decode(const uint8_t* u0p, uint32_t ds0, uint32_t n0, uint32_t* V, uint64_t cap, uint32_t& nv_out,
                        uint32_t* P = nullptr, uint32_t* nm_out = nullptr) {   // P[i]: byte end of value i - ds0; nm: a non-minimal varuint
  const uint32_t l = threadIdx.x % WAVE;
  uint32_t nv = 0;
  bool bad = false;
  for (uint32_t base = ds0; base < n0; base += 16u * WAVE) {
    const uint32_t p0 = base + 16u * l;
    uint32_t T = 0;
    if (p0 < n0) {
      uint4 x; __builtin_memcpy(&x, u0p + p0, 16);   // unaligned (arena tail padding)
      const uint32_t nb = n0 - p0 < 16u ? n0 - p0 : 16u;
      T = ~(hibits8(x.x, x.y) | (hibits8(x.z, x.w) << 8)) & (nb >= 16u ? 0xFFFFu : ((1u << nb) - 1u));
    }
    const uint32_t cnt = (uint32_t)__builtin_popcount(T);
    const uint32_t inc = dpp_incl_add(cnt);
    uint32_t idx = nv + inc - cnt;
    nv += lane63(inc);
    while (T) {
      const uint32_t e = p0 + (uint32_t)__builtin_ctz(T);
      T &= T - 1u;
      const uint32_t w0 = e >= ds0 + 7u ? e - 7u : ds0;   // the 8 bytes [w0, w0 + 8) hold the varuint's last bytes
      uint2 w; __builtin_memcpy(&w, u0p + w0, 8);
      const uint32_t r = e - w0;                          // terminator index in the window
      const uint32_t h = hibits8(w.x, w.y) & ((1u << r) - 1u);
      const uint32_t z = ~h & ((1u << r) - 1u);           // terminators before e in the window
      const uint32_t st = z ? 32u - (uint32_t)__builtin_clz(z) : 0u;
      bad |= (z == 0u && w0 > ds0) || r - st >= 5u;       // >= 9 bytes, or > 5 bytes
      const uint64_t W = ((uint64_t)w.y << 32) | w.x;
      const uint64_t v = pext7(W >> (8u * st), r - st + 1u);
      bad |= v > 0xFFFFFFFFull || idx >= cap;
      if (idx < cap) {
        V[idx] = (uint32_t)v;
        if (P) { P[idx] = e + 1u - ds0; if (r > st && ((W >> (8u * r)) & 0xFFu) == 0u) *nm_out = 1u; }
      }
      idx++;
    }
  }
  nv_out = nv;
  return __ballot(bad) == 0;
}

// A U0 struct the speculative parse could not take, parsed from global memory (rare: kept out of line so
// the chain follow's loop stays small).  Returns end | kind << 32 | failed << 63.
YDEV_NI uint64_t big_skip_global(const uint8_t* u0p, uint32_t n0, uint32_t pos) {
  GCur g; g.init(u0p, n0); g.pos = pos;
  uint32_t kind;
  const bool ok = big_skip<true>(g, kind);
  return (uint64_t)g.pos | ((uint64_t)(kind & 1u) << 32) | (ok ? 0ull : 1ull << 63);
}

// The large-document kernel in two sizes (BigCfg): WAVES waves per workgroup (wave 0 drives, the helper waves join
// the tile, validation, clock-range and delete-set commands through BigCmd), CH tile positions, MAXS / MAXD log
// structs / delete ranges in LDS, SBN block-table entries staged in the tile's LDS during the emit (the rest of the
// tile holds the emit's copy list).  The mid size (4 waves, ~40 KB of LDS: four workgroups per CU) takes every
// large document first and hands one whose log exceeds its LDS to the large size (16 waves, one per CU).
template <int WAVES_, uint32_t CH_, int MAXS_, int MAXD_, uint32_t SBN_>
struct BigCfg {
  static constexpr uint32_t WAVES = WAVES_, THREADS = WAVES_ * 64u, CH = CH_, TILE = CH_ + 64u + 16u, SBN = SBN_;
  static constexpr int MAXS = MAXS_, MAXD = MAXD_;
  static constexpr bool MID = WAVES_ < 16;
  using Tile = BigTileT<CH_>;
  using Lds = BigLdsT<MAXS_, MAXD_>;
  // emit staging in the tile's LDS: [block-table staging (serial emit) | client groups (parallel emit)][splice words][copy list]
  static constexpr uint32_t GCAP = MAXS_ * 3 / 8;
  static constexpr uint32_t SBG = SBN_ * 48u > GCAP * 64u ? SBN_ * 48u : GCAP * 64u;
  static_assert(sizeof(Tile) >= (uint32_t)MAXS_ * sizeof(BigPiece) && sizeof(Tile) >= (uint32_t)MAXD_ * sizeof(BigRange),
                "the log's sort scatters through the tile");
  static_assert(sizeof(Tile) >= SBG + 12 * MAXD_ + 256 * 16 && sizeof(BigBlk) == 48 && sizeof(BigGrp) == 64 && MAXD_ % 4 == 0,
                "emit staging");
};
using BigCfgL = BigCfg<16, 4096, LB_MAXS, LB_MAXD, 256>;
using BigCfgM = BigCfg<4, 1024, 256, 256, 64>;

// ---- the snapshot scan (before k_merge_big, the whole GPU): every byte position p of every large document's U0 parsed
// as a struct start, speculatively -- nx[p] = its end | GC << 31 (0: no parse: not an info byte write_struct emits, a
// Skip, Any arrays / objects or JSON of more than 8 entries, past U0's end), and for parses of at most BIG_VCAP bytes
// vl[p] = its clock length if it is what write_struct emits (big_struct), 0xFFFFFFFF if not (0: not validated).  The
// chain follow in k_merge_big then reads the ends a tile at a time and the validation one word per struct.
#ifndef YGM_BIG_VCAP
#define YGM_BIG_VCAP 64
#endif
constexpr uint32_t BIG_SCAN_CH = 4096, BIG_VCAP = YGM_BIG_VCAP;
struct BigPick { uint64_t pb; uint32_t n0, u0; };   // U0's positions in nx / vl from pb; n0 = 0xFFFFFFFF: not scanned
struct BigScan {
  unsigned long long* cnt;   // [0] positions carved, [1] tasks, [2] / [3] entries of llist / mlist, [4] slow queue
  BigPick* pick;             // per large document (index into fb_list)
  uint2* task;               // (document, chunk of BIG_SCAN_CH positions)
  uint32_t* nv;              // per U0 position (candidates only): big_word
  uint32_t *llist, *mlist;   // fb_list indices by U0 size: over BIG_MID_U0 (the 16-wave size) / the rest (the mid size)
  uint2* vq;                 // slow queue (document, position): candidates k_big_val validates
  uint32_t* pbits;           // per U0 position one bit: a struct whose info byte loses bit 0x20 in the output (documents'
                             // positions start 32-aligned; zeroed by the scan, set by k_merge_big's validation)
  uint64_t ntask_cap, npos_cap, vq_cap;
};
// the scan's word of a U0 position: bits 0-14 the byte length of the struct parsed there (0: no parse, or 32 KB or
// more), bit 15 GC, bits 16-31 its verdict -- the clock length (1 .. 0xFFFE), 0xFFFF refused, 0 none (k_merge_big
// validates it from global memory)
YDEV uint32_t big_v16(uint64_t len, bool ok) { return !ok ? 0xFFFFu : len <= 0xFFFEull ? (uint32_t)len : 0u; }
// U0 bytes past which a document goes to the 16-wave size directly: the mid size walks 1 KB tiles with 4 waves,
// so its time on a snapshot of megabytes (the C3 batch's largest documents) would be the batch's critical path
#ifndef YGM_MID_OCC
#define YGM_MID_OCC 4   // mid-size workgroups per CU the register budget is cut for
#endif
#ifndef YGM_BIG_MID_KB
#define YGM_BIG_MID_KB 512
#endif
constexpr uint32_t BIG_MID_U0 = YGM_BIG_MID_KB * 1024u;
// only a byte write_struct could have emitted as an info byte starts a parse: GC (0) or an Item ref 1..8 without bit 0x20
// next to an origin.  The scan writes nx / vl for these positions only; the follow and the validation test the byte
// before they read them (a struct the chain meets elsewhere is parsed from global memory)
YDEV bool big_cand(uint32_t ib) { const uint32_t rf = ib & 31u; return ib == 0u || (rf >= 1u && rf <= 8u && !((ib & 0xC0u) && (ib & 0x20u))); }
// U0 of each large document (the largest update, the first of equal ones: k_merge_big's rule) and its scan tasks
// (a wave per document, 16 per workgroup: the workgroup carves its positions and tasks with one atomic each)
// A snapshot of many small client blocks (C5: 10 000 blocks of ~100 bytes) over YGM_BIG_SMALLBLK_KB goes to the 16-wave
// size too: its follow steps block to block through the tile's block table, and the 16-wave size's 4 KB tiles cost a
// quarter of the mid size's per-tile work (loads, jump and block tables, validation) per byte.
#ifndef YGM_BIG_SMALLBLK_KB
#define YGM_BIG_SMALLBLK_KB 512
#endif
__global__ __launch_bounds__(1024) void k_big_pick(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                   const uint32_t* __restrict__ doc_upd,
                                                   const uint32_t* __restrict__ fb_list, uint32_t n_fb, BigScan S) {
  __shared__ uint64_t s_pb[16], s_tb[16];
  __shared__ uint32_t s_lg[16], s_lb, s_mb;
  const uint32_t wv = threadIdx.x / WAVE, w = blockIdx.x * 16u + wv, l = threadIdx.x % WAVE;
  uint32_t u0 = 0, n0 = 0, nt = 0;
  if (w < n_fb) {
    const uint32_t d = fb_list[w], ua = doc_upd[d], k = doc_upd[d + 1] - ua;
    uint64_t best = 0;
    for (uint32_t i = l; i < k; i += WAVE) {
      const uint64_t n = upd_off[ua + i + 1] - upd_off[ua + i];
      const uint64_t key = ((n < 0xFFFFFFFFull ? n : 0xFFFFFFFFull) << 32) | (0xFFFFFFFFu - i);
      best = key > best ? key : best;
    }
    for (int o = 32; o > 0; o >>= 1) { const uint64_t x = __shfl_xor(best, o); best = x > best ? x : best; }
    u0 = 0xFFFFFFFFu - (uint32_t)best; n0 = (uint32_t)(best >> 32);
    nt = n0 < 0x7FFFFFFFu ? (n0 + BIG_SCAN_CH - 1u) / BIG_SCAN_CH : 0u;
  }
  bool small_blocks = false;   // U0's block count (its first varuint) against its bytes: blocks of < 256 bytes on average
  if (l == 0 && w < n_fb && n0 > YGM_BIG_SMALLBLK_KB * 1024u && n0 < 0x7FFFFFFFu) {
    const uint8_t* u0p = arena + upd_off[doc_upd[fb_list[w]] + u0];
    uint64_t nb = 0;
    for (uint32_t i = 0, sh = 0; i < 5u; i++, sh += 7) { const uint32_t b = u0p[i]; nb |= (uint64_t)(b & 127u) << sh; if (b < 128u) break; }
    small_blocks = nb * 256ull > (uint64_t)n0;
  }
  if (l == 0) {
    s_pb[wv] = w < n_fb ? ((uint64_t)n0 + 16u + 31u) & ~31ull : 0u; s_tb[wv] = nt;   // (32-aligned: whole pbits words)
    s_lg[wv] = w >= n_fb ? 0u : ((n0 > BIG_MID_U0 || small_blocks) && n0 < 0x7FFFFFFFu) ? 1u : 2u;   // 1: the 16-wave list, 2: the mid list
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // exclusive prefixes over the workgroup's documents, then one carve each
    uint64_t a = 0, b = 0;
    uint32_t nl = 0, nm = 0;
    for (int i = 0; i < 16; i++) {
      const uint64_t x = s_pb[i], y = s_tb[i]; s_pb[i] = a; s_tb[i] = b; a += x; b += y;
      const uint32_t g = s_lg[i]; s_lg[i] = g == 1 ? nl : g == 2 ? nm : 0u; s_lg[i] |= g << 30; nl += g == 1; nm += g == 2;
    }
    const uint64_t pa = atomicAdd(&S.cnt[0], (unsigned long long)a), ta = atomicAdd(&S.cnt[1], (unsigned long long)b);
    s_lb = nl ? (uint32_t)atomicAdd(&S.cnt[2], (unsigned long long)nl) : 0u;
    s_mb = nm ? (uint32_t)atomicAdd(&S.cnt[3], (unsigned long long)nm) : 0u;
    for (int i = 0; i < 16; i++) { s_pb[i] += pa; s_tb[i] += ta; }
  }
  __syncthreads();
  if (w >= n_fb) return;
  if (l == 0) {
    const uint32_t g = s_lg[wv] >> 30, at = s_lg[wv] & 0x3FFFFFFFu;
    if (g == 1) S.llist[s_lb + at] = w; else S.mlist[s_mb + at] = w;
  }
  const uint64_t pb = s_pb[wv], tb = s_tb[wv];
  const bool ok = nt && pb + n0 + 16u <= S.npos_cap && tb + nt <= S.ntask_cap;
  if (l == 0) { BigPick P; P.pb = pb; P.n0 = ok ? n0 : 0xFFFFFFFFu; P.u0 = u0; S.pick[w] = P; }
  if (ok)
    for (uint32_t t = l; t < nt; t += WAVE) S.task[tb + t] = make_uint2(w, t);
}
#ifndef YGM_SCAN_LDS
#define YGM_SCAN_LDS 1
#endif
#ifndef YGM_SCAN_UTF
#define YGM_SCAN_UTF 1   // a candidate string's verdict: 0 the UTF-8 decoder over the stage; 1 ASCII views first (see the scan)
#endif
#ifndef YGM_SCAN_PF
#define YGM_SCAN_PF 1    // parent-form candidates whose parentInfo byte is past 1 are not parsed (see the scan's queue)
#endif
#ifndef YGM_SCAN_CLS
#define YGM_SCAN_CLS 2   // candidate classes queued one after the other (1: position order)
#endif
__global__ __launch_bounds__(256) void k_big_scan(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                  const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ fb_list,
                                                  uint32_t flags, BigScan S) {
  // a wave takes BIG_SCAN_CH / 4 positions of the task, staged in LDS with a margin past them (the structs that start
  // near the end): the candidates (by their byte) are queued, then the lanes parse the queue from LDS -- a lane per
  // candidate, not a lane per position.  A parse that runs into the stage's end is redone from global memory.
  constexpr uint32_t WCH = BIG_SCAN_CH / 4, MARGIN = 256, SQ = (WCH + MARGIN) / 16 + 2;
  __shared__ uint4 s_b[4][SQ];
  __shared__ uint16_t s_q[4][WCH];
  const uint32_t wv = threadIdx.x / WAVE, l = threadIdx.x % WAVE;
  uint16_t* const q = s_q[wv];
  const uint64_t ntask = *(volatile unsigned long long*)&S.cnt[1];
  for (uint64_t t = blockIdx.x; t < ntask; t += gridDim.x) {
    const uint2 T = S.task[t];
    const BigPick P = S.pick[T.x];
    if (P.n0 == 0xFFFFFFFFu) continue;   // (no tasks are carved for such a document)
    const uint8_t* u0p = arena + upd_off[doc_upd[fb_list[T.x]] + P.u0];
    const uint32_t n0 = P.n0, w0 = T.y * BIG_SCAN_CH + wv * WCH;
    if (w0 >= n0) continue;   // (wave-uniform)
    const uint32_t w1 = w0 + WCH < n0 ? w0 + WCH : n0, se = w0 + WCH + MARGIN < n0 ? w0 + WCH + MARGIN : n0;
    if (l < (w1 - w0 + 31u) / 32u) S.pbits[(P.pb + w0) / 32u + l] = 0u;   // (P.pb and w0 are multiples of 32)
    // the stage: the aligned 16-byte chunks holding [w0, se) (a chunk holding a byte of the update is inside the arena)
    const uint8_t* g0 = u0p + w0;
    const uint32_t sh = (uint32_t)((uintptr_t)g0 & 15u), nq = (sh + (se - w0) + 15u) / 16u;
    const uint4* ga = (const uint4*)(g0 - sh);
    for (uint32_t i = l; i < nq; i += WAVE) s_b[wv][i] = ga[i];
    wave_sync();
    const uint8_t* lb = (const uint8_t*)s_b[wv] + sh;   // lb[i] = U0 byte w0 + i
    uint32_t qn = 0;
    // queued by class -- GC and Items with an origin and deleted / string content (text's structs: the verdict from the
    // skip parse) first, then the rest -- so that a wave's lanes parse the same kind of struct more often (the parse
    // branches by kind)
    constexpr uint32_t NCLS = YGM_SCAN_CLS < 1 ? 1u : (uint32_t)YGM_SCAN_CLS;
    for (uint32_t cls = 0; cls < NCLS; cls++)
      for (uint32_t b = 0; b < w1 - w0; b += WAVE) {
        const uint32_t i = b + l;
        const uint32_t ib = i < w1 - w0 ? lb[i] : 1u;
        const bool txt = ib == 0u || ((ib & 0xC0u) && ((ib & 31u) == 1u || (ib & 31u) == 4u));
        const uint32_t k = NCLS == 1u ? 0u : txt ? 0u : (NCLS < 3u || (ib & 0xC0u)) ? 1u : 2u;   // (3: the rest split by origin)
        bool cand = i < w1 - w0 && big_cand(ib) && k == cls;   // (other positions are never read: nothing written)
#if YGM_SCAN_PF
        // a parent-form Item (no origins) whose parentInfo byte is not 0 / 1 is refused by the validation wherever it
        // stands, so it needs no end: its word is 0 (no parse -- the follow parses such a position from global memory
        // should the chain meet it) and the queue keeps the candidates that can be structs write_struct emits
        if (cand && ib != 0u && (ib & 0xC0u) == 0u && i + 1u < se - w0 && lb[i + 1u] > 1u) { cand = false; S.nv[P.pb + w0 + i] = 0u; }
#endif
        const uint64_t m = __ballot(cand);
        if (cand) q[qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = (uint16_t)i;
        qn += (uint32_t)__builtin_popcountll(m);
      }
    wave_sync();
    uint32_t ns = 0;
    for (uint32_t j0 = 0; j0 < qn; j0 += WAVE) {   // (wave-uniform trips: the slow-queue gather is a wave op)
      const uint32_t j = j0 + l, i = j < qn ? q[j] : 0u, p = w0 + i;
      uint32_t e = 0, v = 0;
      bool slow = false;
      if (j < qn) {
#if YGM_SCAN_LDS
        LCur c; c.init((LU8*)lb, se - w0); c.pos = i;   // (LDS-typed reads of the stage)
#else
        GCur c; c.init(lb, se - w0); c.pos = i;
#endif
        uint32_t kind;
        uint64_t cv = 0;
#if YGM_SCAN_SKIP1   // experiment: candidates of the other kinds not parsed (no end: the follow parses them from global memory)
        const uint32_t ib0 = lb[i];
        const bool txt0 = ib0 == 0u || ((ib0 & 0xC0u) && ((ib0 & 31u) == 1u || (ib0 & 31u) == 4u));
        bool ok = txt0 && big_skip(c, kind, 8, &cv) && !c.err;
        if (!txt0) c.err = ST_FALLBACK;
#else
        bool ok = big_skip(c, kind, 8, &cv) && !c.err;
#endif
        const uint8_t* vb = lb;   // (the string's bytes: the stage, or U0 after a redo)
        uint32_t cp = c.pos + w0;
        if (!ok && c.err == ST_MALFORMED && se < n0) {   // ran into the stage's end: the parse again from global memory
          GCur g; g.init(u0p, n0); g.pos = p;
          ok = big_skip(g, kind, 8, &cv) && !g.err;
          cp = g.pos; c.nm = g.nm; vb = u0p;
        }
        if (ok) {
          e = cp - p < 0x8000u ? (cp - p) | (kind == 0 ? 0x8000u : 0u) : 0u;
          const uint32_t info = lb[i], ref = info & 31u;
          if (cp - p <= BIG_VCAP) {
            if (info == 0u || ((info & 0xC0u) && (ref == 1u || ref == 4u))) {
              // GC, or an Item with an origin and deleted / string content (text's structs): big_struct's verdict
              // from the skip parse itself (its varuints minimal, the string strict UTF-8, a non-zero length)
              int64_t len = c.nm ? -1 : (int64_t)cv;
              if (!c.nm && ref == 4u) {
#if YGM_SCAN_UTF == 0 || !YGM_SCAN_LDS
                len = gutf8_u16(vb + (cv >> 32), (uint32_t)cv);
#else
                // the string's bytes from the stage by 8-byte views: all ASCII (the common case, and a cheap no for most
                // of the speculative parses) counts its bytes; otherwise the UTF-8 decoder (1) or no verdict (2: the
                // merge kernel validates it if the chain meets it; 3: experiment, no verdict for any string)
                const uint32_t s0 = (uint32_t)(cv >> 32), sl = (uint32_t)cv;
                bool asc = vb == lb && YGM_SCAN_UTF != 3;
                for (uint32_t k = 0; asc && k < sl; k += 8u) {
                  const uint64_t w = c.w8(s0 + k), m = sl - k >= 8u ? ~0ull : (1ull << (8u * (sl - k))) - 1ull;
                  asc = (w & m & 0x8080808080808080ull) == 0ull;
                }
                len = asc ? (int64_t)sl : YGM_SCAN_UTF == 1 ? gutf8_u16(vb + s0, sl) : -2;
#endif
              }
              v = len == -2 ? 0u : big_v16((uint64_t)len, len > 0 && len < 0xFFFFFFFFll);
            } else {
              // the other kinds: big_struct in k_big_val (its registers would halve this kernel's waves), for a parse
              // whose end could start the next struct (most candidates are bytes inside other structs: their ends
              // land anywhere); the last struct of a block fails this and is validated by k_merge_big
              slow = cp >= se || big_cand(lb[cp - w0]);
            }
          }
        }
      }
      // the slow candidates gather at the queue's front (entries < j0 + 64 are read, entries past it are not yet)
      const uint64_t sm = __ballot(slow);
      if (slow) q[ns + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u))] = (uint16_t)i;
      ns += (uint32_t)__builtin_popcountll(sm);
      if (j < qn) S.nv[P.pb + p] = e | (v << 16);
    }
    if (ns) {   // one append per wave and task (a counter every wave of the grid shares)
      uint64_t base = 0;
      if (l == 0) base = atomicAdd(&S.cnt[4], (unsigned long long)ns);
      base = __shfl(base, 0);
      for (uint32_t k = l; k < ns; k += WAVE)   // (past the queue: v = 0, k_merge_big validates it)
        if (base + k < S.vq_cap) S.vq[base + k] = make_uint2(T.x, w0 + q[k]);
    }
    wave_sync();   // (the queue is rewritten by the next task)
  }
}
// the scan's slow queue: big_struct's verdict for the candidates of other kinds (after k_big_scan, same stream)
// Each lane stages its candidate's bytes -- the aligned 16-byte chunks of [pos, pos + BIG_VCAP] (the queued structs
// parse in at most BIG_VCAP bytes), loads issued together -- into its LDS slot and validates from there: one load
// latency per candidate instead of a chain of dependent window loads through a global-memory cursor.
#ifndef YGM_VAL_LDS
#define YGM_VAL_LDS 1
#endif
#ifndef YGM_VAL_SORT
#define YGM_VAL_SORT 1
#endif
__global__ __launch_bounds__(256) void k_big_val(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                 const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ fb_list,
                                                 uint32_t flags, BigScan S) {
  constexpr uint32_t VW = (BIG_VCAP + 16u + 15u) / 16u;   // 16-byte chunks staged per candidate
  __shared__ uint4 s_w[YGM_VAL_LDS ? 256 : 1][VW];
  const uint64_t nq = *(volatile unsigned long long*)&S.cnt[4], n = nq < S.vq_cap ? nq : S.vq_cap;
#if YGM_VAL_SORT
  // the workgroup's 256 entries are regrouped by their struct's content ref (a counting sort in LDS) before each lane
  // takes one: big_struct branches by content kind, and a wave of mixed kinds runs every branch its lanes take
  __shared__ uint2 s_q[256];
  __shared__ uint16_t s_ix[256];
  __shared__ uint32_t s_cnt[33];
  for (uint64_t b0 = blockIdx.x * 256ull; b0 < n; b0 += gridDim.x * 256ull) {
    const uint32_t t = threadIdx.x;
    if (t < 33u) s_cnt[t] = 0u;
    __syncthreads();
    uint32_t key = 32u, rk = 0;
    if (b0 + t < n) {
      const uint2 Q0 = S.vq[b0 + t];
      s_q[t] = Q0;
      const BigPick P0 = S.pick[Q0.x];
      key = arena[upd_off[doc_upd[fb_list[Q0.x]] + P0.u0] + Q0.y] & 31u;
    }
    rk = atomicAdd(&s_cnt[key], 1u);
    __syncthreads();
    if (t == 0) { uint32_t a = 0; for (uint32_t k = 0; k < 33u; k++) { const uint32_t c = s_cnt[k]; s_cnt[k] = a; a += c; } }
    __syncthreads();
    s_ix[s_cnt[key] + rk] = (uint16_t)t;
    __syncthreads();
    const uint32_t src_t = s_ix[t];
    const uint64_t i = b0 + src_t;
    if (i < n) {
    const uint2 Q = s_q[src_t];
#else
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint2 Q = S.vq[i];
#endif
    const BigPick P = S.pick[Q.x];
    const uint8_t* u0p = arena + upd_off[doc_upd[fb_list[Q.x]] + P.u0];
    const uint32_t wd = S.nv[P.pb + Q.y], end = Q.y + (wd & 0x7FFFu);
#if YGM_VAL_LDS
    const uint8_t* src = u0p + Q.y;
    const uint32_t sh = (uint32_t)((uintptr_t)src & 15u);
    const uint4* g16 = (const uint4*)(src - sh);
    const uint32_t lim = P.n0 - Q.y < VW * 16u - sh ? P.n0 - Q.y : VW * 16u - sh;   // bytes of U0 in the slot
    uint4* slot = s_w[threadIdx.x];
#pragma unroll
    for (uint32_t k = 0; k < VW; k++) {   // (a chunk holding a byte of U0 is inside the arena: its tail padding)
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (16u * k < sh + lim) v = g16[k];
      slot[k] = v;
    }
    LCur w; w.init((LU8*)slot + sh, lim);
    const GStruct g = big_struct(w, flags);
    const bool at_end = w.pos == (wd & 0x7FFFu);
#else
    (void)s_w;
    GCur w; w.init(u0p, P.n0); w.pos = Q.y;
    const GStruct g = big_struct(w, flags);
    const bool at_end = w.pos == end;
#endif
    (void)end;
    S.nv[P.pb + Q.y] = (wd & 0xFFFFu) | (big_v16(g.len, g.ok && !g.patch && at_end && g.len != 0 && g.len < 0xFFFFFFFFull) << 16);
#if YGM_VAL_SORT
    }
    __syncthreads();   // (s_q / s_ix are rewritten by the next round)
#endif
  }
}
// the struct start 2^(k+1) structs after tile position i < BT_CH (k = -1: the next one, from nx), or BJ_NONE
template <class TL>
YDEV uint32_t big_jump(const TL& T, int k, uint32_t i) {
  if (k < 0) { const uint32_t e = T.nx[i]; return e ? (e & 0x7FFFu) : BJ_NONE; }
  return T.jp[k][i];
}
// A client block header (struct count, client, clock: three varuints of <= 5 bytes ending inside the tile)
// from one 16-byte view of the tile: terminators by the top bits, values by 7-bit compaction, nm = a
// non-minimal varuint (a zero last byte).  false: the cursor parse takes it.
YDEV uint32_t big_ctz16(uint32_t t) { return t ? (uint32_t)__builtin_ctz(t) : 16u; }
template <class TL>
YDEV bool big_hdr_fast(const TL& T, uint32_t hp, uint32_t tn, uint64_t& nst, uint64_t& client, uint64_t& clock0,
                       uint32_t& hend, bool& nm) {
  const uint32_t q = hp >> 4, o = hp & 15u, sh = (o & 7u) * 8u;
  const uint4 A = T.b[q], C = T.b[q + 1];
  const uint64_t w0 = ((uint64_t)A.y << 32) | A.x, w1 = ((uint64_t)A.w << 32) | A.z;
  const uint64_t w2 = ((uint64_t)C.y << 32) | C.x, w3 = ((uint64_t)C.w << 32) | C.z;
  const uint64_t a = (o & 8u) ? w1 : w0, b = (o & 8u) ? w2 : w1, c = (o & 8u) ? w3 : w2;
  const uint64_t lo = sh ? (a >> sh) | (b << (64u - sh)) : a, hi = sh ? (b >> sh) | (c << (64u - sh)) : b;
  uint32_t t = ~(hibits8((uint32_t)lo, (uint32_t)(lo >> 32)) | (hibits8((uint32_t)hi, (uint32_t)(hi >> 32)) << 8)) & 0xFFFFu;
  const uint32_t e0 = big_ctz16(t);
  t &= t - 1u;
  const uint32_t e1 = big_ctz16(t);
  t &= t - 1u;
  const uint32_t e2 = big_ctz16(t);
  if (e2 >= 16u || e0 >= 5u || e1 - e0 > 5u || e2 - e1 > 5u || hp + e2 + 1u > tn) return false;
  nst = pext7(dw_at(lo, hi, 0), e0 + 1u);
  client = pext7(dw_at(lo, hi, e0 + 1u), e1 - e0);
  clock0 = pext7(dw_at(lo, hi, e1 + 1u), e2 - e1);
  nm = (e0 > 0u && (dw_at(lo, hi, e0) & 0xFFu) == 0u) || (e1 - e0 > 1u && (dw_at(lo, hi, e1) & 0xFFu) == 0u) ||
       (e2 - e1 > 1u && (dw_at(lo, hi, e2) & 0xFFu) == 0u);
  hend = hp + e2 + 1u;
  return true;
}
#ifndef YGM_BIG_BH
#define YGM_BIG_BH 1
#endif
template <class CF>
YDEV void big_spec(typename CF::Tile& T, const uint8_t* u0p, const uint32_t* nxg, uint32_t at, uint32_t mis, uint32_t n0, uint32_t t0,
                   uint16_t* bh, uint8_t* mk, uint16_t* lst, bool use_bh) {
  // every thread takes the tile positions t0 + j THREADS (t0 < THREADS), their steps interleaved: the loads of one
  // step (global scan words, LDS table entries) are issued together, not as a chain per position
  constexpr uint32_t PER = CF::CH / CF::THREADS;
  static_assert(CF::CH % CF::THREADS == 0, "tile positions split evenly over the workgroup");
  // the scan's struct ends of the tile's positions, tile-relative (an end 32 KB or more away: no entry, the chain
  // follow parses that struct from global memory).  Non-candidate positions hold no word (their load is unused).
  uint32_t rl[PER];   // the ends (block table: marks)
  uint32_t nl = 0;    // the wave's marked positions
  {
    uint32_t v[PER];
    bool c[PER];
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {   // (the position's byte from global memory: loaded with its word and the
                                           //  tile's chunks below, one memory latency for the three)
      const uint32_t i = t0 + j * CF::THREADS;
      const bool in = at + i < n0;
      c[j] = in && big_cand(u0p[at + i]);
      v[j] = in ? nxg[at + i] : 0u;
    }
    {   // the tile's bytes: the aligned 16-byte chunks from U0 byte at - mis (a chunk holding a byte of U0 is inside the
        // arena: its tail padding); read after this call's first barrier
      const uint4* g = (const uint4*)(u0p + at - mis);
      const uint32_t nld = (n0 - at + mis + 15u) / 16u;
      for (uint32_t j = t0; j < CF::TILE / 16 && j < nld; j += CF::THREADS) T.b[j] = g[j];
    }
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t i = t0 + j * CF::THREADS, d = v[j] & 0x7FFFu, rel = i + d;
      const bool e = c[j] && d && rel < 0x8000u;
      T.nx[i] = (uint16_t)(e ? rel | (v[j] & 0x8000u) : 0u);
      rl[j] = e ? rel : 0x8000u;
      if (use_bh) { mk[i] = i == 0u; bh[i] = BJ_NONE; }   // (the tile's origin: the chain's entry, a block header in a run)
    }
  }
#ifdef YGM_DIAG
  unsigned long long dgs0 = DIAG_NOW();
  auto dgs = [&](int i) { if (threadIdx.x == 0) { const unsigned long long n_ = DIAG_NOW(); atomicAdd(&ygm_diag[29 + i], n_ - dgs0); dgs0 = n_; } };
#else
  auto dgs = [](int) {};
#endif
  // a table lookup (level k, -1: nx) without a branch: the read clamped into the tile, BJ_NONE for s >= CH (the
  // levels unrolled, so the level's table is a constant offset)
  auto bj = [&](int k, uint32_t s) -> uint32_t {
    const uint32_t sc = s < CF::CH ? s : 0u;
    uint32_t v;
    if (k < 0) { const uint32_t e = T.nx[sc]; v = e ? (e & 0x7FFFu) : BJ_NONE; }
    else v = T.jp[k][sc];
    return s < CF::CH ? v : BJ_NONE;
  };
  // jump tables by doubling (every thread of the workgroup calls this, so the barriers match)
#pragma unroll
  for (int k = 0; k < BJ_LV; k++) {
    __syncthreads();
    uint32_t a[PER];
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) a[j] = bj(k - 1, t0 + j * CF::THREADS);
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) T.jp[k][t0 + j * CF::THREADS] = (uint16_t)bj(k - 1, a[j]);
    if (k == 0 && use_bh) {   // marks: the positions a struct of the tile ends at -- a block header starts at one of them
                              // (right after its previous block's last struct) or at the tile's origin
#pragma unroll
      for (uint32_t j = 0; j < PER; j++)
        if (rl[j] < CF::CH) mk[rl[j]] = 1;
    }
    if (k == 1 && use_bh) {   // (the marks landed at this level's barrier) the wave's marked positions, compacted into its
                              // own segment of lst: the table is computed for them only, a lane each, not for every
                              // position with most lanes idle
#pragma unroll
      for (uint32_t j = 0; j < PER; j++) {
        const uint32_t i = t0 + j * CF::THREADS;
        const bool m = mk[i] != 0 && at + i < n0;
        const uint64_t b = __ballot(m);
        if (m) lst[(t0 / WAVE) * (WAVE * PER) + nl + lanes_below(b)] = (uint16_t)i;
        nl += (uint32_t)__popcll(b);
      }
    }
    if (k == 0) dgs(0);
  }
  if (!YGM_BIG_BH || !use_bh) { dgs(1); return; }   // (documents of large blocks: the table would not be used, C3)
  // the block table: bh[i] = the tile position right after the whole client block whose header would start at tile
  // position i (the header decoded from the tile, then its nst structs jumped through the tables along the bits of
  // nst), or BJ_NONE (no header parse, nst 0 or >= 64, a struct without a table entry or starting past the tile's CH
  // positions).  The chain follow then steps from block to block with one lookup each.
  __syncthreads();
  dgs(1);
  const uint32_t tn = n0 - (at - mis) < CF::TILE ? n0 - (at - mis) : CF::TILE;
  for (uint32_t e = t0 % WAVE; e < nl; e += WAVE) {
    const uint32_t i = lst[(t0 / WAVE) * (WAVE * PER) + e];
    uint64_t nst = 0, cl, ck;
    uint32_t he = 0;
    bool nm;
    if (big_hdr_fast(T, mis + i, tn, nst, cl, ck, he, nm) && nst != 0u && nst < 64u) {
      uint32_t S = he - mis;
#pragma unroll
      for (int k = 0; k < 6; k++) {
        const uint32_t x = bj(k - 1, S);
        S = ((nst >> k) & 1u) ? x : S;
      }
      bh[i] = (uint16_t)S;
    }
  }
  dgs(2);
}
// after a tile's spec (cmd 1): the helper waves touch the next tile's bytes and both tiles' scan words, a load per
// 128-byte line, so that wave 0's loads of them after its chain follow (the next spec, this tile's verdicts) hit L2
template <uint32_t CH, uint32_t NT>
YDEV void big_prefetch(const BigCmd& C, uint32_t t0) {
  const uint32_t a = C.at, n0 = C.n0;
  const uint32_t b0 = a + CH < n0 ? a + CH : n0, b1 = a + 2u * CH + 128u < n0 ? a + 2u * CH + 128u : n0;
  const uint32_t nb = (b1 - b0 + 127u) / 128u, nw = (b1 - a + 31u) / 32u;
  uint32_t acc = 0;
  for (uint32_t i = t0; i < nb + nw; i += NT) acc ^= i < nb ? (uint32_t)C.u0p[b0 + i * 128u] : C.aux[a + (i - nb) * 32u];
  asm volatile("" ::"v"(acc));   // (the loads are the point)
}
// the U0 walk's struct records [vs, ns) (rec, written by the follow without lengths): the scan's verdict (its word,
// C.aux) where it has one, else validated from global memory; stored with their clock lengths.  True if any is not
// what write_struct emits.  Run once at the walk's end by the whole workgroup: off the follow's serial chain, with
// the global parses of every lane in flight together.
// Returns bit 0: some struct is not what write_struct emits; bit 1: some struct is, once its info byte loses bit 0x20
// (marked in the document's bitmap pbits: C.at = its first word; the emit's copies clear the bit).
template <uint32_t NT>
YDEV uint32_t big_validate(BigRec* rec, const BigCmd& C, uint32_t flags, uint32_t t0, uint32_t* pbits_all) {
  uint32_t r = 0;
  uint32_t* const pbits = pbits_all + C.at;
  for (uint64_t i = C.vs + t0; i < C.ns; i += NT) {
    BigRec R = rec[C.sbase + i];
    const uint32_t v16 = big_cand(C.u0p[R.start]) ? C.aux[R.start] >> 16 : 0u;   // (the scan wrote candidate positions only)
    uint64_t len = v16 == 0xFFFFu ? 0xFFFFFFFFull : v16;
    if (len == 0u) {   // (the scan's end for R.start, when it has one, is R.end: the chain took it from nx)
      GCur w; w.init(C.u0p, C.n0); w.pos = R.start;
      const GStruct g = big_struct(w, flags);
      len = g.ok && w.pos == R.end ? g.len : 0u;
      if (len && g.patch) { atomicOr(&pbits[R.start >> 5], 1u << (R.start & 31u)); r |= 2u; }
    }
    r |= (len == 0u || len >= 0xFFFFFFFFull) ? 1u : 0u;
    rec[C.sbase + i].len = (uint32_t)len;
  }
  return r;
}

// ---- U0's delete set spliced instead of streamed (big documents: U0's delete set large against the log's ranges).
// Scratch words of the document: V [0, W3) values, P [W3, 2 W3) each value's byte end (from the delete set's start),
// then the entry table: for entry e (a client of U0's delete set, descending) eidx[e] (index of its client value in V),
// eclient, en (range count), ebs / ebe (bytes of the whole entry), then a bitmap of the client values' indices.
struct BigDsPlan { uint32_t C, end, b0, bend; bool fast; };   // b0 / bend: bytes of the entries (from the delete set's start)
YDEV uint32_t* ds_eclient(uint32_t* eidx, uint32_t C) { return eidx + C; }
YDEV uint32_t* ds_en(uint32_t* eidx, uint32_t C) { return eidx + 2u * C; }
YDEV uint32_t* ds_ebs(uint32_t* eidx, uint32_t C) { return eidx + 3u * C; }
YDEV uint32_t* ds_ebe(uint32_t* eidx, uint32_t C) { return eidx + 4u * C; }
YDEV uint32_t* ds_bits(uint32_t* eidx, uint32_t C) { return eidx + 5u * C; }
// the client entries (wave 0, the walk is a chain: entry e + 1 starts 2 + 2 n values after entry e); false: not
// spliceable (truncated, an empty or repeated client, clients not descending, no room)
YDEV bool big_ds_entries(const uint32_t* V, uint32_t dsn, uint32_t* eidx, uint64_t w3, BigDsPlan& DP) {
  const uint32_t l = threadIdx.x % WAVE;
  const uint32_t ncl = V[0];
  if ((uint64_t)ncl * 5u + dsn / 32u + 8u > w3 || 4ull * ncl + 1u > dsn) return false;
  uint32_t idx = 1, prevc = 0, wb = 0xFFFFFFFFu, wv = 0;   // V[wb + j] in lane j
  for (uint32_t c = 0; c < ncl; c++) {
    if (idx + 1u >= dsn) return false;
    if (wb == 0xFFFFFFFFu || idx < wb || idx + 1u >= wb + (uint32_t)WAVE) { wb = idx; wv = wb + l < dsn ? V[wb + l] : 0u; }
    const uint32_t client = (uint32_t)__builtin_amdgcn_readlane((int)wv, (int)(idx - wb));
    const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)wv, (int)(idx + 1u - wb));
    if (n == 0u || (c && client >= prevc) || (uint64_t)idx + 2u + 2ull * n > dsn) return false;
    if (l == 0) { eidx[c] = idx; ds_eclient(eidx, ncl)[c] = client; ds_en(eidx, ncl)[c] = n; }
    prevc = client;
    idx += 2u + 2u * n;
  }
  DP.C = ncl; DP.end = idx;
  return true;
}
// cmd 4, the whole workgroup: the client bitmap, each entry's byte bounds, then every range canonical -- non-empty,
// inside 32-bit clocks, and starting after the previous range of its entry ends (sorted, disjoint, not adjacent: the
// union would write it as it is).  Range starts are the odd value indices that are not client values (entries start
// at odd indices: 1, then + 2 + 2 n).  C: vs = V, ns = eidx, sbase = W3, n0 = entries, at = end of the entries.
template <uint32_t NT>
YDEV bool big_ds_canon(const BigCmd& C, uint32_t t0) {
  const uint32_t* V = (const uint32_t*)(uintptr_t)C.vs;
  const uint32_t* P = V + C.sbase;
  uint32_t* eidx = (uint32_t*)(uintptr_t)C.ns;
  const uint32_t ne = C.n0, end = C.at, nw = end / 32u + 1u;
  uint32_t* bits = ds_bits(eidx, ne);
  for (uint32_t w = t0; w < nw; w += NT) bits[w] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __syncthreads();
  for (uint32_t e = t0; e < ne; e += NT) {
    const uint32_t i = eidx[e];
    atomicOr(&bits[i / 32u], 1u << (i % 32u));
    ds_ebs(eidx, ne)[e] = P[i - 1u];
    ds_ebe(eidx, ne)[e] = P[i + 1u + 2u * ds_en(eidx, ne)[e]];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __syncthreads();
  auto is_client = [&](uint32_t j) { return (bits[j / 32u] >> (j % 32u)) & 1u; };
  bool ok = true;
  for (uint32_t j = 3u + 2u * t0; j < end; j += 2u * NT) {
    if (is_client(j)) continue;
    const uint64_t k = V[j], len = V[j + 1u];
    ok &= len != 0u && k + len <= 0xFFFFFFFFull;
    if (!is_client(j - 2u)) ok &= k > (uint64_t)V[j - 2u] + V[j - 1u];
  }
  return ok;
}
// each log range against U0's entry of its client (wave 0, a lane per range): the entry by binary search over the
// clients (ent: the first entry at or after its client; bit 31 set when U0 has none for it), then the U0 ranges it merges with: [a, b1) = the ranges ending at or after its start and starting at or
// before its end (U0's ranges are disjoint and not adjacent: both bounds by binary search)
// X (LDS, 3 x maxd words): per range the byte start of entry `ent` (the delete set's end if none) and, when U0 has
// its client, that entry's range count and byte end -- what the emit's sequential loop reads, staged ahead
YDEV void big_ds_plan(const uint32_t* V, const uint32_t* P, uint32_t* eidx, BigDsPlan& DP, BigRange* rg, uint32_t nrg,
                      uint32_t* X, uint32_t maxd) {
  const uint32_t l = threadIdx.x % WAVE, ne = DP.C;
  const uint32_t* ecl = ds_eclient(eidx, ne);
  DP.b0 = P[0]; DP.bend = P[DP.end - 1u];
  for (uint32_t r = l; r < nrg; r += WAVE) {
    BigRange& R = rg[r];
    const uint32_t client = 0xFFFFFFFFu - (uint32_t)(R.key >> 32), k = (uint32_t)R.key, ke = k + R.len;
    uint32_t lo = 0, hi = ne;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (ecl[m] > client) lo = m + 1u; else hi = m; }
    R.ent = lo | 0x80000000u; R.a = 0; R.b1 = 0; R.s = k; R.e = ke; R.pa = 0; R.pb = 0;   // (bit 31: no entry)
    if (lo < ne && ecl[lo] == client) {
      const uint32_t i0 = eidx[lo] + 2u, n = ds_en(eidx, ne)[lo];
      uint32_t a = 0, h = n;
      while (a < h) { const uint32_t m = (a + h) >> 1; if ((uint64_t)V[i0 + 2u * m] + V[i0 + 2u * m + 1u] < k) a = m + 1u; else h = m; }
      uint32_t b1 = a; h = n;
      while (b1 < h) { const uint32_t m = (b1 + h) >> 1; if (V[i0 + 2u * m] <= ke) b1 = m + 1u; else h = m; }
      if (a < b1) {
        const uint32_t ka = V[i0 + 2u * a], eb = V[i0 + 2u * (b1 - 1u)] + V[i0 + 2u * (b1 - 1u) + 1u];
        R.s = ka < k ? ka : k; R.e = eb > ke ? eb : ke;
      }
      R.ent = lo; R.a = a; R.b1 = b1; R.pa = P[i0 + 2u * a - 1u]; R.pb = P[i0 + 2u * b1 - 1u];
      X[maxd + r] = n; X[2u * maxd + r] = ds_ebe(eidx, ne)[lo];
    }
    X[r] = lo < ne ? ds_ebs(eidx, ne)[lo] : DP.bend;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  wave_sync();
}

// ---- the parallel struct emit (wave 0, lanes over log pieces / client groups; U0's block headers all minimal).
// A client group is the log pieces of one client (sorted by clock) and U0's block of that client if it has one
// ("touched"); the U0 block goes in before the first piece at or after its clock.  Every other U0 block is copied as
// written, in runs between groups.  The plan (pass 0) sizes every piece (a Skip over a gap to its predecessor, then its
// bytes), every group (header, pieces, the U0 block) and places every group by an exclusive scan of what each changes
// against U0's bytes; pass 1 writes headers and Skips from the lanes and queues every copy on the copy list.
YDEV int64_t wave_incl_add_i64(int64_t v) {
  const uint32_t l = threadIdx.x % WAVE;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) { const int64_t t = __shfl_up(v, o, WAVE); if (l >= (uint32_t)o) v += t; }
  return v;
}
YDEV void big_put_vu(uint8_t* d, uint64_t v) {   // one lane writes a varuint
  while (v > 127) { *d++ = (uint8_t)(0x80u | (v & 127)); v >>= 7; }
  *d = (uint8_t)v;
}
// the predecessor of piece q in its group: the U0 block when it goes right before q, else piece q - 1 (none for the
// group's first piece); returns whether there is one
template <class LDS>
YDEV bool big_piece_pred(const LDS& L, const BigGrp& R, uint32_t q, uint32_t& pend, bool& pgc) {
  if ((R.flags & 1u) && R.uslot == q) { pend = R.clock1; pgc = (R.flags & 4u) != 0; return true; }
  if (q > R.q0) { const BigPiece& P = L.pc[q - 1]; pend = (uint32_t)P.key + P.len; pgc = P.gc(); return true; }
  return false;
}
// plan: 0 planned, 1 outside the class (overlap / GC junction: the document defers), 2 not planned (more client groups
// than G holds: the serial emit takes it).  ngr groups, nbo output blocks, sbytes bytes of the structs part.
template <class LDS>
YDEV int big_plan_structs(LDS& L, BigGrp* G, uint32_t gcap, const BigBlk* T, uint32_t nb, uint32_t npc, uint32_t S0, uint32_t ds0,
                          uint32_t& ngr_out, uint64_t& nbo, uint64_t& sbytes) {
  const uint32_t l = threadIdx.x % WAVE;
  // 1. the groups: runs of one client among the sorted pieces
  uint32_t ngr = 0;
  for (uint32_t cb = 0; cb < npc; cb += WAVE) {
    const uint32_t q = cb + l;
    const bool in = q < npc;
    const uint32_t X = in ? (uint32_t)(L.pc[q].key >> 32) : 0u;
    const bool gs = in && (q == 0 || (uint32_t)(L.pc[q - 1].key >> 32) != X);
    const bool ge = in && (q + 1 == npc || (uint32_t)(L.pc[q + 1].key >> 32) != X);
    const uint64_t m = __ballot(gs);
    const uint32_t gi = ngr + lanes_below(m) + (gs ? 1u : 0u) - 1u;
    ngr += (uint32_t)__builtin_popcountll(m);
    if (in && gi < gcap) {
      L.pc[q].gi = gi;
      if (gs) { G[gi].q0 = q; G[gi].uslot = 0xFFFFFFFFu; G[gi].cnt = 0; }
      if (ge) G[gi].qend = q + 1u;
    }
  }
  ngr_out = ngr;
  if (ngr > gcap) return 2;
  wave_sync();
  // 2. each group against the block table: the first block at or below its client (binary search, blocks descending)
  for (uint32_t g = l; g < ngr; g += WAVE) {
    BigGrp& R = G[g];
    const uint64_t client = 0xFFFFFFFFull - (uint32_t)(L.pc[R.q0].key >> 32);
    uint32_t lo = 0, hi = nb;
    while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (T[md].client > client) lo = md + 1u; else hi = md; }
    R.flags = 0; R.nst = 0; R.clock0 = R.clock1 = R.b0 = R.b1 = 0; R.h0ins = ds0;
    if (lo < nb) {
      const BigBlk B = T[lo];
      R.h0ins = B.h0;
      if (B.client == client) {
        R.flags = 1u | (B.first_gc ? 2u : 0u) | (B.last_gc ? 4u : 0u);
        R.nst = B.nst; R.clock0 = (uint32_t)B.clock0; R.clock1 = (uint32_t)B.clock1; R.b0 = B.b0; R.b1 = B.b1;
      }
    }
  }
  wave_sync();
  // 3. the U0 block's slot: before the first piece at or after its clock
  for (uint32_t cb = 0; cb < npc; cb += WAVE) {
    const uint32_t q = cb + l;
    if (q < npc) {
      BigGrp& R = G[L.pc[q].gi];
      const uint32_t c0 = (uint32_t)L.pc[q].key;
      if ((R.flags & 1u) && c0 >= R.clock0 && (q == R.q0 || (uint32_t)L.pc[q - 1].key < R.clock0)) R.uslot = q;
    }
  }
  wave_sync();
  for (uint32_t g = l; g < ngr; g += WAVE) if (G[g].uslot == 0xFFFFFFFFu) G[g].uslot = G[g].qend;
  wave_sync();
  // 4. pieces: the Skip over the gap to the predecessor; output bytes and structs; inclusive byte prefix
  bool bad = false;
  uint32_t carry = 0;
  for (uint32_t cb = 0; cb < npc; cb += WAVE) {
    const uint32_t q = cb + l;
    uint32_t bq = 0;
    if (q < npc) {
      const BigPiece& P = L.pc[q];
      BigGrp& R = G[P.gi];
      const uint32_t c0 = (uint32_t)P.key;
      uint32_t pend = 0; bool pgc = false;
      uint32_t gap = 0;
      if (big_piece_pred(L, R, q, pend, pgc)) {
        bad |= c0 < pend || (c0 == pend && pgc && P.gc());
        gap = c0 > pend ? c0 - pend : 0u;
      }
      bq = P.nb() + (gap ? 1u + vu_len(gap) : 0u);
      atomicAdd(&R.cnt, gap ? 2u : 1u);
    }
    const uint32_t inc = dpp_incl_add(bq) + carry;
    if (q < npc) L.pc[q].pre = inc;
    carry = lane63(inc);
  }
  wave_sync();
  // 5. groups: the U0 block's gap, header, size; placement by an exclusive scan of each group's change in bytes
  int64_t dcarry = 0;
  uint32_t nlog = 0;
  for (uint32_t gb = 0; gb < ngr; gb += WAVE) {
    const uint32_t g = gb + l;
    int64_t delta = 0;
    if (g < ngr) {
      BigGrp& R = G[g];
      const bool touched = (R.flags & 1u) != 0;
      const uint32_t q0 = R.q0, qe = R.qend, us = R.uslot;
      const uint32_t pb0 = q0 ? L.pc[q0 - 1].pre : 0u;
      uint32_t gapu = 0;
      if (touched && us > q0) {
        const BigPiece& P = L.pc[us - 1];
        const uint32_t c1 = (uint32_t)P.key + P.len;
        bad |= R.clock0 < c1 || (R.clock0 == c1 && P.gc() && (R.flags & 2u));
        gapu = R.clock0 > c1 ? R.clock0 - c1 : 0u;
      }
      const uint32_t cnt = R.cnt + (touched ? R.nst + (gapu ? 1u : 0u) : 0u);
      const uint32_t first = (touched && us == q0) ? R.clock0 : (uint32_t)L.pc[q0].key;
      const uint32_t client = 0xFFFFFFFFu - (uint32_t)(L.pc[q0].key >> 32);
      const uint32_t hdr = vu_len(cnt) + vu_len(client) + vu_len(first);
      const uint32_t gapub = gapu ? 1u + vu_len(gapu) : 0u;
      const uint64_t bytes = (uint64_t)hdr + (L.pc[qe - 1].pre - pb0) + (touched ? (uint64_t)(R.b1 - R.b0) + gapub : 0u);
      R.cnt = cnt; R.first = first; R.gapu = gapu; R.hdr = hdr;
      R.upos = hdr + ((us > q0 ? L.pc[us - 1].pre : pb0) - pb0) + gapub;
      delta = (int64_t)bytes - (touched ? (int64_t)(R.b1 - R.h0ins) : 0);
      nlog += touched ? 0u : 1u;
    }
    const int64_t inc = wave_incl_add_i64(delta);
    if (g < ngr) G[g].rel = (uint32_t)((int64_t)(G[g].h0ins - S0) + dcarry + inc - delta);
    dcarry += __shfl(inc, WAVE - 1, WAVE);
  }
  wave_sync();
  for (int o = 32; o > 0; o >>= 1) nlog += (uint32_t)__shfl_xor((int)nlog, o, WAVE);
  nbo = (uint64_t)nb + nlog;
  sbytes = (uint64_t)((int64_t)(ds0 - S0) + dcarry);
  return __ballot(bad) ? 1 : 0;
}
// pass 1: the structs part at out + base (after the block count)
template <class LDS>
YDEV void big_write_structs(const LDS& L, const BigGrp* G, uint32_t ngr, uint32_t npc, const uint8_t* u0p, const uint8_t* arena,
                            uint32_t S0, uint32_t ds0, uint64_t sbytes, uint64_t base, BigOut& o) {
  const uint32_t l = threadIdx.x % WAVE;
  uint8_t* const ob = o.o + base;
  // U0's untouched blocks in runs between groups, and the touched blocks' struct bytes
  uint32_t a = S0;
  for (uint32_t g = 0; g < ngr; g++) {
    const BigGrp& R = G[g];
    if (R.h0ins > a) o.add((uint64_t)(uintptr_t)(u0p + a), base + R.rel - (R.h0ins - a), R.h0ins - a);
    if (R.flags & 1u) { o.add((uint64_t)(uintptr_t)(u0p + R.b0), base + R.rel + R.upos, R.b1 - R.b0); a = R.b1; }
    else a = R.h0ins;
  }
  if (ds0 > a) o.add((uint64_t)(uintptr_t)(u0p + a), base + sbytes - (ds0 - a), ds0 - a);
  // group headers, and the Skip before a touched block
  for (uint32_t g = l; g < ngr; g += WAVE) {
    const BigGrp& R = G[g];
    uint8_t* d = ob + R.rel;
    const uint32_t client = 0xFFFFFFFFu - (uint32_t)(L.pc[R.q0].key >> 32);
    big_put_vu(d, R.cnt); d += vu_len(R.cnt);
    big_put_vu(d, client); d += vu_len(client);
    big_put_vu(d, R.first);
    if (R.gapu) { uint8_t* s = ob + R.rel + R.upos - (1u + vu_len(R.gapu)); *s = 10; big_put_vu(s + 1, R.gapu); }
  }
  // pieces: the Skip from the lane, the bytes through the copy list (one entry per piece, appended in parallel)
  o.le = ~0ull;   // (no merging with the entries above)
  for (uint32_t cb = 0; cb < npc; cb += WAVE) {
    if (o.nc + WAVE > o.cap) o.flush();
    const uint32_t q = cb + l;
    const bool in = q < npc;
    uint64_t dst = 0;
    if (in) {
      const BigPiece& P = L.pc[q];
      const BigGrp& R = G[P.gi];
      const uint32_t pb0 = R.q0 ? L.pc[R.q0 - 1].pre : 0u;
      uint32_t off = R.hdr + ((q > R.q0 ? L.pc[q - 1].pre : pb0) - pb0);
      if ((R.flags & 1u) && q >= R.uslot) off += (R.gapu ? 1u + vu_len(R.gapu) : 0u) + (R.b1 - R.b0);
      dst = base + R.rel + off;
      uint32_t pend = 0; bool pgc = false;
      if (big_piece_pred(L, R, q, pend, pgc) && (uint32_t)P.key > pend) {
        const uint32_t gap = (uint32_t)P.key - pend;
        o.o[dst] = 10; big_put_vu(o.o + dst + 1, gap); dst += 1u + vu_len(gap);
      }
    }
    const uint64_t m = __ballot(in);
    if (in) { BigCp E; E.src = (uint64_t)(uintptr_t)(arena + L.pc[q].src); E.dst = (uint32_t)dst; E.n = L.pc[q].nb(); o.cl[o.nc + lanes_below(m)] = E; }
    o.nc += (uint32_t)__builtin_popcountll(m);
  }
  o.le = ~0ull;
}

// ---- the parallel splice emit of the delete set (wave 0; after big_ds_plan).  Lanes over the sorted log ranges find
// the client starts and the merge groups (a range starts a group when it starts beyond the running maximum end of its
// client's earlier ranges: a segmented max scan), fold each group's end / last touched U0 range onto its first range,
// and add per client (LDS atomics) its groups, their span bytes and the U0 ranges / bytes they absorb.  One short serial
// loop over the log clients places them (the untouched entries before each go out as one verbatim run); the lanes then
// write headers and spans and queue every verbatim run / segment on the copy list.  W: LDS words, 7 per log client + 1
// per range; false (capacity): the serial emit takes it.  Range flags in BigRange.len (free after big_ds_plan): bit 0
// client start, bit 1 group start, bits 2-12 client ordinal, 13-23 the range's group start.
YDEV uint32_t big_u64max_scan(uint64_t& v) {   // inclusive max scan of v over the wave (in place); returns nothing useful
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) { const uint64_t t = __shfl_up(v, o, WAVE); if ((threadIdx.x % WAVE) >= (uint32_t)o) v = t > v ? t : v; }
  return 0;
}
template <class LDS>
YDEV bool big_ds_par(LDS& L, const BigDsPlan& DP, const uint32_t* X, uint32_t maxd, uint32_t nrg, uint32_t* W, uint32_t wcap,
                     const uint8_t* dsb, BigOut& o, uint64_t& nc) {
  const uint32_t l = threadIdx.x % WAVE, ne = DP.C;
  if (nrg > 2047u) return false;
  if (3ull * nrg > wcap) return false;
  uint32_t* const PR = W;                                   // per range: running max end (steps 1-2), contribution scan (5)
  uint32_t* const PRB = W + nrg;                            // ... running max of b1 and pb within the client (steps 1-2):
  uint32_t* const PRP = W + 2u * nrg;                       //     not monotone (a short range inside a long one absorbs less)
  // 1. flags, client ordinals, group starts
  uint32_t nci = 0, gcarry = 0;
  uint64_t mcarry = 0, bcarry = 0, pcarry = 0;
  for (uint32_t cb = 0; cb < nrg; cb += WAVE) {
    const uint32_t r = cb + l;
    const bool in = r < nrg;
    const uint32_t X0 = in ? (uint32_t)(L.rg[r].key >> 32) : 0u;
    const bool cs = in && (r == 0 || (uint32_t)(L.rg[r - 1].key >> 32) != X0);
    const uint64_t m = __ballot(cs);
    const uint32_t ci = nci + lanes_below(m) + (cs ? 1u : 0u) - 1u;
    nci += (uint32_t)__builtin_popcountll(m);
    uint64_t v = in ? (((uint64_t)ci << 32) | L.rg[r].e) : 0ull;
    big_u64max_scan(v);
    v = v > mcarry ? v : mcarry;
    uint64_t ex = __shfl_up(v, 1, WAVE);
    if (l == 0) ex = mcarry;
    const bool gs = in && (cs || (uint32_t)(ex >> 32) != ci || L.rg[r].s > (uint32_t)ex);
    uint64_t gv = gs ? r : 0u;
    big_u64max_scan(gv);
    const uint32_t gsi = (uint32_t)gv > gcarry ? (uint32_t)gv : gcarry;
    uint64_t vb = in ? (((uint64_t)ci << 32) | L.rg[r].b1) : 0ull, vp = in ? (((uint64_t)ci << 32) | L.rg[r].pb) : 0ull;
    big_u64max_scan(vb); big_u64max_scan(vp);
    vb = vb > bcarry ? vb : bcarry; vp = vp > pcarry ? vp : pcarry;
    if (in) { L.rg[r].len = (cs ? 1u : 0u) | (gs ? 2u : 0u) | (ci << 2) | (gsi << 13); PR[r] = (uint32_t)v; PRB[r] = (uint32_t)vb; PRP[r] = (uint32_t)vp; }
    mcarry = __shfl(v, WAVE - 1, WAVE); bcarry = __shfl(vb, WAVE - 1, WAVE); pcarry = __shfl(vp, WAVE - 1, WAVE);
    gcarry = (uint32_t)__builtin_amdgcn_readlane((int)gsi, WAVE - 1);
  }
  if (nci > 2047u || 7ull * nci + 3ull * nrg > wcap) return false;
  uint32_t* const CW = W + 3u * nrg;                        // per log client: ng, span bytes, absorbed ranges, absorbed bytes, first range, offset, untouched run
  for (uint32_t i = l; i < 7u * nci; i += WAVE) CW[i] = 0u;
  wave_sync();
  // 2. each group's end (the running maximum at its last range) and last absorbed U0 range onto its first range
  for (uint32_t cb = 0; cb < nrg; cb += WAVE) {
    const uint32_t r = cb + l;
    uint32_t g = 0, ge = 0, b1 = 0, pb = 0; bool last = false;
    if (r < nrg) {
      last = r + 1 == nrg || (L.rg[r + 1].len & 2u);
      g = L.rg[r].len >> 13; ge = PR[r]; b1 = PRB[r]; pb = PRP[r];
    }
    wave_sync();
    if (last) { L.rg[g].e = ge; L.rg[g].b1 = b1; L.rg[g].pb = pb; }
    wave_sync();
  }
  // 3. per client sums (LDS atomics) at the group starts
  for (uint32_t cb = 0; cb < nrg; cb += WAVE) {
    const uint32_t r = cb + l;
    if (r < nrg) {
      const BigRange& R = L.rg[r];
      const uint32_t f = R.len, ci = (f >> 2) & 0x7FFu;
      if (f & 1u) CW[7u * ci + 4u] = r;
      if (f & 2u) {
        const bool touched = !(R.ent >> 31);
        atomicAdd(&CW[7u * ci + 0u], 1u);
        atomicAdd(&CW[7u * ci + 1u], vu_len(R.s) + vu_len(R.e - R.s));
        if (touched) { atomicAdd(&CW[7u * ci + 2u], R.b1 - R.a); atomicAdd(&CW[7u * ci + 3u], R.pb - R.pa); }
      }
    }
  }
  wave_sync();
  // 4. the log clients in order (serial, a few operations each): records placed after the untouched entries before them
  uint64_t off = 0;
  uint32_t cur = DP.b0, eu = 0;
  nc = 0;
  for (uint32_t c = 0; c < nci; c++) {
    uint32_t* w = CW + 7u * c;
    const uint32_t r0 = w[4];
    const BigRange& R = L.rg[r0];
    const uint32_t lo = R.ent & 0x7FFFFFFFu;
    const bool touched = !(R.ent >> 31);
    const uint32_t xbs = X[r0];
    const uint32_t U = xbs - cur;
    const uint32_t client = 0xFFFFFFFFu - (uint32_t)(R.key >> 32);
    const uint32_t n = touched ? X[maxd + r0] : 0u, be = touched ? X[2u * maxd + r0] : 0u;
    const uint32_t nruns = n - w[2] + w[0];
    const uint64_t verb = touched ? (uint64_t)(be - xbs - vu_len(client) - vu_len(n)) - w[3] : 0u;
    if (l == 0) { w[5] = (uint32_t)off; w[6] = U; }
    off += (uint64_t)U + vu_len(client) + vu_len(nruns) + w[1] + verb;
    nc += (lo - eu) + 1u;
    cur = touched ? be : xbs; eu = touched ? lo + 1u : lo;
  }
  const uint32_t tail = DP.bend - cur;
  nc += ne - eu;
  if (!o.w) { o.n += off + tail; return true; }
  // 5. writes at o.o + base: client headers and untouched runs (lanes over clients), spans and segments (lanes over
  //    ranges: a group's place in its client is an exclusive scan of what each group writes -- the U0 bytes between the
  //    previous group and it, then its span)
  const uint64_t base = o.n;
  wave_sync();
  o.flush();
  o.le = ~0ull;
  uint32_t carry = 0;
  for (uint32_t cb = 0; cb < nrg; cb += WAVE) {
    const uint32_t r = cb + l;
    uint32_t contrib = 0;
    if (r < nrg && (L.rg[r].len & 2u)) {
      const BigRange& R = L.rg[r];
      const uint32_t ci = (R.len >> 2) & 0x7FFu;
      uint32_t seg = 0;
      if (!(R.ent >> 31)) {
        const uint32_t* w = CW + 7u * ci;
        const uint32_t r0 = w[4];
        const uint32_t client = 0xFFFFFFFFu - (uint32_t)(R.key >> 32), n = X[maxd + r0];
        const uint32_t prevpb = (R.len & 1u) ? X[r0] + vu_len(client) + vu_len(n) : L.rg[L.rg[r - 1].len >> 13].pb;
        seg = R.pa - prevpb;
      }
      contrib = seg + vu_len(R.s) + vu_len(R.e - R.s);
    }
    const uint32_t inc = dpp_incl_add(contrib) + carry;
    if (r < nrg) PR[r] = inc - contrib;                      // exclusive scan
    carry = lane63(inc);
  }
  wave_sync();
  for (uint32_t cb = 0; cb < nrg; cb += WAVE) {
    if (o.nc + 3u * WAVE > o.cap) o.flush();
    const uint32_t r = cb + l;
    // up to three copies per lane: the client's untouched run (A), the U0 bytes before a group (B), after the last (C)
    BigCp A, B, C; A.n = B.n = C.n = 0u;
    if (r < nrg) {
      const BigRange& R = L.rg[r];
      const uint32_t f = R.len, ci = (f >> 2) & 0x7FFu;
      const uint32_t* w = CW + 7u * ci;
      const uint32_t r0 = w[4];
      const bool touched = !(R.ent >> 31);
      const uint32_t client = 0xFFFFFFFFu - (uint32_t)(R.key >> 32);
      const uint32_t n = touched ? X[maxd + r0] : 0u;
      const uint32_t nruns = n - w[2] + w[0];
      const uint64_t body = base + w[5] + w[6] + vu_len(client) + vu_len(nruns);   // after the client's header
      if (f & 1u) {   // the client's untouched run and header; for a touched entry the U0 bytes after its last group
        if (w[6]) { A.src = (uint64_t)(uintptr_t)(dsb + X[r0] - w[6]); A.dst = (uint32_t)(base + w[5]); A.n = w[6]; }
        uint8_t* h = o.o + base + w[5] + w[6];
        big_put_vu(h, client); big_put_vu(h + vu_len(client), nruns);
        if (touched) {
          uint32_t rl = r0;   // the client's last range, and its last group (start gl)
          while (rl + 1 < nrg && !(L.rg[rl + 1].len & 1u)) rl++;
          const uint32_t gl = L.rg[rl].len >> 13;
          const BigRange& G = L.rg[gl];
          const uint32_t prevpb = (G.len & 1u) ? X[r0] + vu_len(client) + vu_len(n) : L.rg[L.rg[gl - 1].len >> 13].pb;
          const uint64_t endw = (uint64_t)(PR[gl] - PR[r0]) + (G.pa - prevpb) + vu_len(G.s) + vu_len(G.e - G.s);
          const uint32_t be = X[2u * maxd + r0];
          if (be > G.pb) { C.src = (uint64_t)(uintptr_t)(dsb + G.pb); C.dst = (uint32_t)(body + endw); C.n = be - G.pb; }
        }
      }
      if (f & 2u) {   // the group: the U0 bytes since the previous group, then its span
        uint32_t seg = 0, prevpb = 0;
        if (touched) {
          prevpb = (f & 1u) ? X[r0] + vu_len(client) + vu_len(n) : L.rg[L.rg[r - 1].len >> 13].pb;
          seg = R.pa - prevpb;
        }
        const uint64_t at = body + (PR[r] - PR[r0]);
        if (seg) { B.src = (uint64_t)(uintptr_t)(dsb + prevpb); B.dst = (uint32_t)at; B.n = seg; }
        uint8_t* h = o.o + at + seg;
        big_put_vu(h, R.s); big_put_vu(h + vu_len(R.s), R.e - R.s);
      }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const BigCp& E = k == 0 ? A : k == 1 ? B : C;
      const uint64_t m = __ballot(E.n != 0u);
      if (E.n) o.cl[o.nc + lanes_below(m)] = E;
      o.nc += (uint32_t)__builtin_popcountll(m);
    }
  }
  if (tail) o.add((uint64_t)(uintptr_t)(dsb + cur), base + off, tail);
  o.le = ~0ull;
  o.n = base + off + tail;
  return true;
}

// block clock ranges [vs, ns) of the block table (cmd 3, the whole workgroup): clock0 + the validated lengths of
// the block's struct records; true if one passes 2^32 - 1
template <uint32_t NT>
YDEV bool big_clock_ranges(BigBlk* blk, const BigRec* rec, const BigCmd& C, uint32_t t0) {
  bool bad = false;
  for (uint64_t b = C.vs + t0; b < C.ns; b += NT) {
    const uint32_t nst = blk[b].nst, s0 = blk[b].s0;
    uint64_t clk = blk[b].clock0;
    for (uint32_t q = 0; q < nst; q++) clk += rec[C.sbase + s0 + q].len;
    bad |= clk > 0xFFFFFFFFull;
    blk[b].clock1 = clk;
  }
  return bad;
}

template <class CF>
__global__ __launch_bounds__(CF::THREADS, CF::MID ? YGM_MID_OCC : 1) void k_merge_big(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                    const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ fb_list,
                                                    uint32_t flags, uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                                                    uint64_t* __restrict__ out_len, int32_t* __restrict__ status, DocMeta* meta,
                                                    uint32_t* __restrict__ fb2_list, BigBlk* __restrict__ blk, uint64_t blk_cap,
                                                    BigRec* __restrict__ rec, uint64_t rec_cap, uint64_t slot_total, uint64_t out_cap,
                                                    BigScan S, const uint32_t* __restrict__ fbx, uint32_t* __restrict__ up_list) {
  __shared__ typename CF::Lds L;
  __shared__ typename CF::Tile T0;
  __shared__ unsigned long long s_pick;
  __shared__ uint64_t s_base, s_sbase, s_ds0, s_at;
  __shared__ BigCmd s_cmd;
  __shared__ uint32_t s_rst[CF::CH / 2], s_ren[CF::CH / 2];   // byte ranges of the current tile's structs (>= 2 bytes each)
  constexpr uint32_t SBQ = CF::MID ? 24u : 64u;   // block records staged in LDS before a store (mid: room for s_bh)
  __shared__ BigBlk s_blk[SBQ];
  __shared__ uint32_t s_cpre[WAVE];
  __shared__ uint16_t s_bh[YGM_BIG_BH ? CF::CH : 1];   // the tile's block table (big_spec)
  __shared__ uint8_t s_mk[YGM_BIG_BH ? CF::CH : 1];    // ... computed at these positions only
  __shared__ uint16_t s_hl[WAVE + 2];                  // a run of blocks found from it: their tile positions
#ifndef YGM_BIG_ROT
#define YGM_BIG_ROT 0
#endif
  // the logical thread index: the chain-follow wave (logical wave 0) is physical wave blockIdx.x % WAVES, so the
  // followers of the mid size's workgroups sharing a CU do not all land on one SIMD (they are latency chains: four on
  // one SIMD share its issue while the helpers' SIMDs idle)
  const uint32_t tid = YGM_BIG_ROT && CF::MID ? (threadIdx.x + CF::THREADS - WAVE * (blockIdx.x % CF::WAVES)) % CF::THREADS
                                              : threadIdx.x;
  if (!CF::MID && threadIdx.x == 0) atomicAdd(&meta->big_started, 1u);   // (k_big_wait holds the mid size back until then)
  if (tid >= WAVE) {   // helper waves: wave 0's tile commands until it sends 0 (one barrier pair per command)
    for (;;) {
      __syncthreads();
      const BigCmd C = s_cmd;
      if (C.cmd == 0) return;
      if (C.cmd == 1) big_spec<CF>(T0, C.u0p, C.aux, C.at, C.mis, C.n0, tid, s_bh, s_mk, (uint16_t*)s_rst, C.tb != 0u);
      else if (C.cmd == 3) { if (big_clock_ranges<CF::THREADS>(blk, rec, C, tid)) L.bad = 1; }
      else if (C.cmd == 4) { if (!big_ds_canon<CF::THREADS>(C, tid)) s_cmd.tb = 1; }
      else if (C.cmd == 6) {
        big_rank_sort<BigPiece, CF::THREADS>(L.pc, (uint32_t)C.vs, (BigPiece*)&T0, tid);
        big_rank_sort<BigRange, CF::THREADS>(L.rg, (uint32_t)C.ns, (BigRange*)&T0, tid);
      }
      else if (C.cmd == 5) big_copy_chunks(const_cast<uint8_t*>(C.u0p), (const BigCp*)(uintptr_t)C.vs, (uint32_t)C.ns, s_cpre, C.tb,
                                           (tid / WAVE) * 4u * WAVE, CF::WAVES * 4u * WAVE, C.aux, (const uint8_t*)(uintptr_t)C.sbase, C.n0);
      else { const uint32_t r = big_validate<CF::THREADS>(rec, C, flags, tid, S.pbits); if (r & 1u) L.bad = 1; if (r & 2u) L.patch = 1; }
      __syncthreads();
      if (C.cmd == 1) big_prefetch<CF::CH, CF::THREADS - WAVE>(C, tid - WAVE);   // (while wave 0 follows the chain)
    }
  }
  const uint32_t l = tid;
  DIAGL_T0
  const uint32_t w = fbx ? fbx[blockIdx.x] : blockIdx.x;   // index into fb_list (and the scan's picks)
  const uint32_t d = fb_list[w];
  const uint32_t ua = doc_upd[d], k = doc_upd[d + 1] - ua;
  if (l == 0) { L.npc = 0; L.nrg = 0; L.bad = (flags & 2u) ? 1u : 0u; L.patch = 0; s_pick = 0; }   // YGM_F_FORCE_SEQ: all to the sequential kernel
  wave_sync();
  // ---- the snapshot U0: the largest update (the first of equal ones)
  for (uint32_t i = l; i < k; i += WAVE) {
    const uint64_t n = upd_off[ua + i + 1] - upd_off[ua + i];
    if (n >= 0xFFFFFFFFull) L.bad = 1;
    atomicMax(&s_pick, ((unsigned long long)(n < 0xFFFFFFFFull ? n : 0xFFFFFFFFull) << 32) | (0xFFFFFFFFu - i));
  }
  wave_sync();
  const uint32_t U0 = 0xFFFFFFFFu - (uint32_t)s_pick;
  // ---- log updates, lanes in parallel: every struct a piece, every delete range a record.  The log's bytes are
  //      staged in the tile's LDS first (free before the U0 walk; one copy list for the wave, its loads in flight
  //      together) when they fit, and parsed there: from global memory each update is a chain of dependent loads.
  constexpr uint32_t LG_LIST = 256, LG_CAP = (uint32_t)sizeof(typename CF::Tile) - LG_LIST * (uint32_t)sizeof(BigCp);
  uint8_t* const lstage = (uint8_t*)&T0;
  BigCp* const llist = (BigCp*)(lstage + LG_CAP);
  uint32_t lbytes = 0;
  bool staged = k >= 2u && k - 1u <= LG_LIST;
  for (uint32_t i0 = 0; staged && i0 < k; i0 += WAVE) {   // stage offsets: an exclusive scan of the sizes (U0's: 0)
    const uint32_t i = i0 + l;
    const uint64_t sz = i < k && i != U0 ? upd_off[ua + i + 1] - upd_off[ua + i] : 0ull;
    const uint32_t s32 = sz < LG_CAP ? (uint32_t)sz : LG_CAP;
    const uint32_t inc = dpp_incl_add(s32);
    if (i < k && i != U0) { BigCp E; E.src = (uint64_t)(uintptr_t)(arena + upd_off[ua + i]); E.dst = lbytes + inc - s32; E.n = s32; llist[i < U0 ? i : i - 1u] = E; }
    lbytes += lane63(inc);
    staged = lbytes <= LG_CAP && __ballot(sz >= LG_CAP) == 0;
  }
  if (staged) big_copy_list(lstage, llist, k - 1u, s_cpre);   // (wave-synchronous)
  auto walk = [&](auto& c, uint64_t a) {
    bool bad = false;
    const uint64_t nb = c.vu();
    uint64_t prevc = ~0ull;
    for (uint64_t b = 0; b < nb && !c.err && !bad; b++) {
      const uint64_t nst = c.vu(), client = c.vu();
      uint64_t clock = c.vu();
      // blocks in descending client order in every input (otherwise yjs's writer can revisit a client)
      bad |= client > 0xFFFFFFFFull || client >= prevc;
      prevc = client;
      for (uint64_t q = 0; q < nst && !c.err && !bad; q++) {
        const uint32_t b0 = c.pos;
        const GStruct g = big_struct(c, flags);
        bad |= !g.ok || g.patch || g.len == 0 || clock + g.len > 0xFFFFFFFFull;   // (a log struct to patch: the general path)
        if (bad) break;
        const uint32_t slot = atomicAdd(&L.npc, 1u);
        if (slot < (uint32_t)CF::MAXS) {
          BigPiece& P = L.pc[slot];
          P.key = ((uint64_t)(0xFFFFFFFFu - (uint32_t)client) << 32) | clock;
          P.len = (uint32_t)g.len; P.src = a + b0; P.nbg = (c.pos - b0) | (g.kind == 0 ? 0x80000000u : 0u);
        }
        clock += g.len;
      }
    }
    const uint64_t nc = c.vu();
    for (uint64_t q = 0; q < nc && !c.err && !bad; q++) {
      const uint64_t client = c.vu(), nr = c.vu();
      for (uint64_t r = 0; r < nr && !c.err && !bad; r++) {
        const uint64_t ck = c.vu(), ln = c.vu();
        bad |= client > 0xFFFFFFFFull || ck + ln > 0xFFFFFFFFull;
        if (bad) break;
        const uint32_t slot = atomicAdd(&L.nrg, 1u);
        if (slot < (uint32_t)CF::MAXD) { L.rg[slot].key = ((uint64_t)(0xFFFFFFFFu - (uint32_t)client) << 32) | ck; L.rg[slot].len = (uint32_t)ln; }
      }
    }
    if (bad || c.err) L.bad = 1;
  };
  for (uint32_t i = l; i < k; i += WAVE) {
    if (i == U0) continue;
    const uint64_t a = upd_off[ua + i];
    const uint32_t n = (uint32_t)(upd_off[ua + i + 1] - a);
    if (staged) { const BigCp E = llist[i < U0 ? i : i - 1u]; LCur c; c.init((LU8*)(lstage + E.dst), n); walk(c, a); }
    else { GCur c; c.init(arena + a, n); walk(c, a); }
  }
  DIAGL(0);
  wave_sync();
  if (CF::MID && !L.bad && (L.npc > (uint32_t)CF::MAXS || L.nrg > (uint32_t)CF::MAXD)) {   // the large size takes it
    if (l == 0) { s_cmd.cmd = 0; up_list[atomicAdd(&meta->mid_defer, 1u)] = w; }
    __syncthreads();   // (the helper waves' first barrier: they read cmd 0 and leave)
    return;
  }
  // ---- U0, tile by tile (BigTile): the wave stages CF::CH + BT_OV bytes in LDS with aligned 16-byte
  //      loads; every lane parses a struct speculatively (skip-only: end and kind) at each of its
  //      positions of the first CF::CH bytes; the chain of real struct boundaries is then followed
  //      with one LDS lookup per struct (block headers parsed from the tile), every struct's byte
  //      range recorded; before the tile moves on, the wave validates its structs in parallel from LDS.
  //      A struct the speculative parse could not take (leaves the tile, JSON of > 8 entries) is parsed from
  //      global memory; a struct failing validation in the tile is validated again from global memory.
  const uint8_t* u0p = arena + upd_off[ua + U0];
  const uint32_t n0 = (uint32_t)(upd_off[ua + U0 + 1] - upd_off[ua + U0]);
  const uint64_t ncap = n0 + 1u;                            // structs take >= 2 bytes; delete-set values >= 1
  const BigPick PK = S.pick[w];
  const uint32_t* const nxg = S.nv + PK.pb;                 // the scan's words (ends and verdicts) of U0's positions
  if (l == 0 && (PK.n0 != n0 || PK.u0 != U0)) L.bad = 1;   // (not scanned: the sequential kernel takes it)
  wave_sync();
  uint64_t base = 0, sbase = 0, nb = 0, NS = 0;
  uint32_t S0 = 0;                                         // U0 position of the first block (after the block count)
  bool acanon = true;                                      // every block header minimal (the parallel emit's condition)
  // tile origin tc0 (U0 position), tb = tc0 rounded down to a 16-byte aligned address: LDS byte j of
  // the tile is U0 byte tb + j, so tile cursors run in tile coordinates (pointers stay inside T0)
  uint32_t tc0 = 0, tb = 0, tn = 0;                        // tn: tile cursor end (tile coordinates)
  [[maybe_unused]] uint64_t dg_spec = 0, dg_val = 0;       // diagnostic build: time in the speculative parse / validation
  DIAG_C(uint64_t dc_blk = 0, dc_step = 0, dc_st = 0, dc_glob = 0, dc_hslow = 0;)   // ... and follow counts
  DIAG_C(uint64_t dt_hdr = 0, dt_st = 0, dt_tail = 0, dt_tile = 0;)                   // ... and follow time by part
  const uint8_t* const tp = (const uint8_t*)T0.b;
  bool use_bh = false;   // the block table pays for documents of small blocks (C5: 10 000 blocks in <= 1.3 MB)
  auto load_tile = [&](uint32_t at, bool spec) {
    const uint32_t mis = (uint32_t)((uintptr_t)(u0p + at) & 15u);
    const uint4* g = (const uint4*)(u0p + at - mis);
    const uint32_t nld = (n0 - at + mis + 15u) / 16u;     // aligned chunks up to the end of U0 (arena tail padding)
    wave_sync();                                           // readers of the previous tile are done
    tc0 = at; tb = at - mis;
    tn = n0 - tb < CF::TILE ? n0 - tb : CF::TILE;
    if (!spec) {   // (the spec loads the tile with its scan words)
      for (uint32_t j = l; j < CF::TILE / 16 && j < nld; j += WAVE) T0.b[j] = g[j];
      wave_sync();
      return;
    }
    const uint64_t dg0 = DIAG_NOW();
    if (l == 0) { s_cmd.cmd = 1; s_cmd.at = at; s_cmd.mis = mis; s_cmd.n0 = n0; s_cmd.aux = nxg; s_cmd.u0p = u0p; s_cmd.tb = use_bh ? 1u : 0u; }
    __syncthreads();
    big_spec<CF>(T0, u0p, nxg, at, mis, n0, l, s_bh, s_mk, (uint16_t*)s_rst, use_bh);
    __syncthreads();
    dg_spec += DIAG_NOW() - dg0;
  };
  uint64_t vs = 0;                                         // first struct record not yet validated
  // the tile's struct records [vs, NS) (LDS) go to rec without lengths (wave 0, no barrier): they are validated once,
  // at the walk's end (cmd 2)
  auto validate = [&]() {
    wave_sync();
    for (uint64_t i = vs + l; i < NS; i += WAVE) { BigRec R; R.start = s_rst[i - vs]; R.end = s_ren[i - vs]; R.len = 0; rec[sbase + i] = R; }
    vs = NS;
    wave_sync();
  };
  auto validate_all = [&]() {
    const uint64_t dg0 = DIAG_NOW();
    if (l == 0) {
      s_cmd.cmd = 2; s_cmd.vs = 0; s_cmd.ns = NS; s_cmd.sbase = sbase; s_cmd.u0p = u0p; s_cmd.n0 = n0; s_cmd.aux = nxg;
      s_cmd.at = (uint32_t)(PK.pb / 32u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // the records before every wave reads them
    __syncthreads();
    { const uint32_t r = big_validate<CF::THREADS>(rec, s_cmd, flags, l, S.pbits); if (r & 1u) L.bad = 1; if (r & 2u) L.patch = 1; }
    __syncthreads();
    dg_val += DIAG_NOW() - dg0;
  };
  if (!L.bad) {
    GCur c; c.init(u0p, n0);
    bool bad = false;
    nb = c.vu();
    use_bh = YGM_BIG_BH && nb * 256ull > (uint64_t)n0;   // (average block under 256 bytes)
    if (l == 0) { s_base = atomicAdd(&meta->big_cursor, (unsigned long long)nb); s_sbase = atomicAdd(&meta->big_scur, (unsigned long long)ncap); }
    wave_sync();
    base = s_base; sbase = s_sbase;
    bad |= c.err || nb > n0 / 4u + 1u || base + nb > blk_cap || sbase + ncap > rec_cap;
    uint32_t pos = c.pos;
    S0 = pos;
    bool have = false;
    uint64_t prevc = ~0ull;
    uint32_t bq = 0;                                       // blocks staged in s_blk
    auto flush_blk = [&](uint64_t upto) {                  // s_blk holds blocks [upto - bq, upto)
      wave_sync();
      const uint4* src = (const uint4*)s_blk;
      uint4* dst = (uint4*)(blk + base + upto - bq);
      for (uint32_t u = l; u < bq * (uint32_t)(sizeof(BigBlk) / 16); u += WAVE) dst[u] = src[u];
      bq = 0;
      wave_sync();
    };
    for (uint64_t b = 0; b < nb && !bad;) {
      DIAG_C(const uint64_t dq0 = DIAG_NOW();)
      if (!have || pos >= tc0 + CF::CH) { if (have) validate(); load_tile(pos, true); have = true; }
      DIAG_C(const uint64_t dq1 = DIAG_NOW(); dt_tile += dq1 - dq0;)
      if (YGM_BIG_BH && use_bh) {
        // ---- a run of whole blocks from the tile's block table (big_spec): lane 0 chains their header positions, one
        //      LDS lookup per block; the lanes then decode the headers and record the structs, a block each
        const uint32_t cap = SBQ - bq < (uint32_t)WAVE ? SBQ - bq : (uint32_t)WAVE;
        const uint32_t lim = nb - b < (uint64_t)cap ? (uint32_t)(nb - b) : cap;
        if (l == 0) {
          uint32_t p = pos - tc0, nh = 0;
          while (nh < lim && p < CF::CH) {
            const uint32_t e = s_bh[p];
            if (e == BJ_NONE) break;
            s_hl[nh++] = (uint16_t)p; p = e;
          }
          s_hl[WAVE] = (uint16_t)nh; s_hl[WAVE + 1] = (uint16_t)p;
        }
        wave_sync();
        const uint32_t nh = s_hl[WAVE], pend = s_hl[WAVE + 1];
        if (nh) {
          const bool on = l < nh;
          const uint32_t hp = on ? (uint32_t)s_hl[l] : 0u, mis = tc0 - tb;   // (tile coordinates: mis + relative position)
          uint64_t hn = 0, hc = 0, hk = 0;
          uint32_t he = mis;
          bool hnm = false;
          const bool okh = on && big_hdr_fast(T0, mis + hp, tn, hn, hc, hk, he, hnm);
          const uint32_t nst = okh ? (uint32_t)hn : 0u;   // (1 .. 63: the table's condition)
          const uint32_t inc = dpp_incl_add(nst), ex = inc - nst, tot = lane63(inc);
          const uint32_t r0 = (uint32_t)(NS - vs) + ex;
          uint32_t S = he - mis, fg = 0, lg = 0;
          for (uint32_t q = 0; q < nst; q++) {   // (every struct start of the block is < CH: the table's condition)
            const uint32_t E = T0.nx[S];
            s_rst[r0 + q] = tc0 + S; s_ren[r0 + q] = tc0 + (E & 0x7FFFu);
            if (q == 0) fg = (E >> 15) & 1u;
            lg = (E >> 15) & 1u;
            S = E & 0x7FFFu;
          }
          // client blocks strictly descending (from the block before the run), clients < 2^32
          const uint32_t plo = (uint32_t)__shfl_up((int)(uint32_t)hc, 1u, WAVE), phi = (uint32_t)__shfl_up((int)(uint32_t)(hc >> 32), 1u, WAVE);
          const uint64_t hprev = l == 0 ? prevc : (((uint64_t)phi << 32) | plo);
          bad |= __ballot(on && (!okh || hc >= hprev || hc > 0xFFFFFFFFull)) != 0;
          acanon &= __ballot(on && hnm) == 0;
          if (on) {
            BigBlk& B = s_blk[bq + l];
            B.nst = nst; B.client = hc; B.clock0 = hk; B.clock1 = 0;
            B.h0 = tc0 + hp; B.hcanon = !hnm; B.pad = 0; B.b0 = he + tb; B.s0 = (uint32_t)(NS + ex);
            B.b1 = tc0 + S; B.first_gc = (uint8_t)fg; B.last_gc = (uint8_t)lg;
          }
          const uint32_t ql = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hc, (int)nh - 1);
          const uint32_t qh = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(hc >> 32), (int)nh - 1);
          prevc = ((uint64_t)qh << 32) | ql;
          NS += tot; b += nh; bq += nh;
          pos = tc0 + pend;
          DIAG_C(dc_blk += nh; dc_st += tot;)
          if (bq == SBQ) flush_blk(b);
          continue;
        }
      }
      uint64_t hn, hc, hk;
      uint32_t he;
      bool hnm;
      DIAG_C(dc_blk++;)
      if (!big_hdr_fast(T0, pos - tb, tn, hn, hc, hk, he, hnm)) {
        DIAG_C(dc_hslow++;)
        GCur h; h.init(tp, tn); h.pos = pos - tb; h.nm = 0;
        hn = h.vu(); hc = h.vu(); hk = h.vu();
        bad |= h.err != 0;
        he = h.pos; hnm = h.nm != 0;
      }
      // the block record goes to its LDS staging slot now (nothing of it stays live across the struct loop)
      const uint32_t bnst = (uint32_t)hn;
      bad |= bnst == 0 || hc >= prevc || hc > 0xFFFFFFFFull;
      prevc = hc;
      const uint32_t h0 = pos;
      pos = he + tb;
      if (l == 0) {
        BigBlk& B = s_blk[bq];
        B.nst = bnst; B.client = hc; B.clock0 = hk; B.clock1 = 0;
        B.h0 = h0; B.hcanon = !hnm; B.pad = 0; B.b0 = pos; B.s0 = (uint32_t)NS;
      }
      acanon &= !hnm;
      uint32_t fgc = 0, lgc = 0;
      DIAG_C(const uint64_t dq2 = DIAG_NOW(); dt_hdr += dq2 - dq1;)
      for (uint32_t q = 0; q < bnst && !bad;) {
        if (pos >= tc0 + CF::CH) { validate(); load_tile(pos, true); }
        // up to 64 of the block's structs per step: lane j finds the start of struct q + j by composing
        // the jump tables along the bits of j; the structs taken are the leading lanes that start inside
        // the tile and have a speculative parse
        const uint32_t want = bnst - q < 64u ? bnst - q : 64u;
        uint32_t S = pos - tc0;
#pragma unroll
        for (int k = 0; k < 6; k++) {   // (branch-free: the reads clamped into the tile, every level; lanes past want
                                        //  have no use for theirs, the bits of those below it select)
          const uint32_t sc = S < CF::CH ? S : 0u;
          uint32_t x;
          if (k == 0) { const uint32_t e = T0.nx[sc]; x = e ? (e & 0x7FFFu) : BJ_NONE; }
          else x = T0.jp[k - 1][sc];
          S = (((l >> k) & 1u) && S < CF::CH) ? x : S;
        }
        const uint32_t E = (l < want && S < CF::CH) ? (uint32_t)T0.nx[S] : 0u;
        const uint64_t tk = __ballot(E != 0u);
        const uint32_t m = ~tk ? (uint32_t)__builtin_ctzll(~tk) : 64u;
        if (m) {
          // lane id and record index recomputed here: a loop-invariant record address would be hoisted,
          // spilled, and its reload would wait on every store in flight
          uint32_t li;
          asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(li));
          const uint32_t nr = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(NS - vs));
          if (li < m) { s_rst[nr + li] = tc0 + S; s_ren[nr + li] = tc0 + (E & 0x7FFFu); }
          const uint32_t E0 = (uint32_t)__builtin_amdgcn_readlane((int)E, 0), El = (uint32_t)__builtin_amdgcn_readlane((int)E, (int)m - 1);
          if (q == 0) fgc = (E0 >> 15) & 1u;
          lgc = (El >> 15) & 1u;
          NS += m; q += m;
          DIAG_C(dc_step++; dc_st += m;)
          pos = tc0 + (El & 0x7FFFu);
          continue;
        }
        // the struct at pos has no speculative parse: parsed from global memory
        const uint64_t r = big_skip_global(u0p, n0, pos);
        DIAG_C(dc_glob++;)
        bad |= (r >> 63) != 0;
        const uint32_t kind = (uint32_t)(r >> 32) & 1u, end = (uint32_t)r;
        if (l == 0) { s_rst[NS - vs] = pos; s_ren[NS - vs] = end; }
        if (q == 0) fgc = kind == 0;
        lgc = kind == 0;
        NS++; q++;
        pos = end;
      }
      DIAG_C(const uint64_t dq3 = DIAG_NOW(); dt_st += dq3 - dq2;)
      if (!bad) {   // staged in LDS, stored SBQ at a time (a store per block would be waited on by the next block's loads)
        if (l == 0) { BigBlk& B = s_blk[bq]; B.b1 = pos; B.first_gc = (uint8_t)fgc; B.last_gc = (uint8_t)lgc; }
        if (++bq == SBQ) flush_blk(b + 1);
      }
      b++;
      DIAG_C(dt_tail += DIAG_NOW() - dq3;)
    }
    if (!bad && bq) flush_blk(nb);
    if (have && !bad) { validate(); validate_all(); }
    const uint32_t ds0 = pos;
    // U0's delete set must already be in union order (client descending, clock ascending): checked by
    // the emit's first pass, which streams it anyway
    wave_sync();
    if (l == 0) { s_ds0 = ds0; if (bad) L.bad = 1; }
  }
#ifndef YGM_DIAG_BIGDS
  DIAG_PUT(6, dg_spec); DIAG_PUT(7, dg_val);
  DIAG_C(if (l == 0) { atomicAdd(&ygm_diag[16], (unsigned long long)dc_blk); atomicAdd(&ygm_diag[17], (unsigned long long)dc_step);
                       atomicAdd(&ygm_diag[18], (unsigned long long)dc_st); atomicAdd(&ygm_diag[19], (unsigned long long)dc_glob);
                       atomicAdd(&ygm_diag[20], (unsigned long long)dc_hslow);
                       atomicAdd(&ygm_diag[25], dt_tile); atomicAdd(&ygm_diag[26], dt_hdr); atomicAdd(&ygm_diag[27], dt_st);
                       atomicAdd(&ygm_diag[28], dt_tail); })
#endif
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // validated lengths before the clock-range pass
  wave_sync();
  if (!L.bad) {
    // block clock ranges, the whole workgroup: clock0 + the lengths of the block's structs
    if (l == 0) { s_cmd.cmd = 3; s_cmd.vs = base; s_cmd.ns = base + nb; s_cmd.sbase = sbase; }
    __syncthreads();
    if (big_clock_ranges<CF::THREADS>(blk, rec, s_cmd, l)) L.bad = 1;
    __syncthreads();
  }
  // ---- U0's delete set as values V (the struct records' scratch is free after the clock-range pass), with each
  //      value's byte end P (big_ds_decode, wave 0).  When it is large against the log's ranges it is SPLICED
  //      (BigDsPlan): its client entries walked once (wave 0), every range checked canonical -- client-descending
  //      entries, sorted, disjoint and non-adjacent non-empty ranges, minimal varuints: what the union would write
  //      for it -- by the whole workgroup (cmd 4); each log range then finds the U0 ranges it merges with by binary
  //      search, and the emit copies everything else verbatim.  Otherwise the emit's passes stream it range by range.
  uint32_t* const dsv = (uint32_t*)(rec + sbase);
  const uint64_t dW3 = ncap * (sizeof(BigRec) / 4) / 3;      // V | P | entries + client bitmap, dW3 words each
  uint32_t* const dsp = dsv + dW3;
  uint32_t* const eidx = dsv + 2 * dW3;                       // entry e: index of its client value in V
  uint32_t dsn = 0;
  BigDsPlan DP; DP.C = 0; DP.end = 0; DP.fast = false;
  // (wave 0 alone until cmd 4: the helper waves wait at their loop's first barrier, so every barrier below pairs with
  //  one of theirs -- the command's two and big_ds_canon's own)
  if (!L.bad) {
    uint32_t nm = 0;
    const bool ok = big_ds_decode(u0p, (uint32_t)s_ds0, n0, dsv, dW3, dsn, dsp, &nm);
    const bool any_nm = __ballot(nm != 0u) != 0;
    if (!ok && l == 0) L.bad = 1;
    DP.fast = ok && !any_nm && !(flags & 1u);
    if (DP.fast) DP.fast = big_ds_entries(dsv, dsn, eidx, dW3, DP);
    if (DP.fast) {   // every range of every entry canonical (the whole workgroup); a failure streams instead
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // the entry table before the helper waves read it
      if (l == 0) {
        s_cmd.cmd = 4; s_cmd.vs = (uint64_t)(uintptr_t)dsv; s_cmd.ns = (uint64_t)(uintptr_t)eidx; s_cmd.sbase = dW3;
        s_cmd.n0 = DP.C; s_cmd.at = DP.end; s_cmd.tb = 0;
      }
      __syncthreads();
      const BigCmd C4 = s_cmd;                                 // (copied before big_ds_canon's first barrier: tb is
      if (!big_ds_canon<CF::THREADS>(C4, l)) s_cmd.tb = 1;                  //  written after its last; every writer writes 1)
      __syncthreads();
      DP.fast = s_cmd.tb == 0;
    }
  }
  DIAG_C(if (l == 0) { atomicAdd(&ygm_diag[21], 1ull); atomicAdd(&ygm_diag[22], DP.fast ? 1ull : 0ull);
                       atomicAdd(&ygm_diag[23], (unsigned long long)dsn); atomicAdd(&ygm_diag[24], (unsigned long long)DP.C); })
  // (the helper waves stay in their command loop: the emit's copy lists are run by every wave, cmd 5)
  DIAGL(1);
  const uint32_t npc = L.npc, nrg = L.nrg;
  bool bad = L.bad || npc > (uint32_t)CF::MAXS || nrg > (uint32_t)CF::MAXD;
  if (!bad) {   // cmd 6: the log's pieces and ranges sorted by the whole workgroup (the tile's LDS, free now, as scratch)
    if (l == 0) { s_cmd.cmd = 6; s_cmd.vs = npc; s_cmd.ns = nrg; }
    __syncthreads();
    big_rank_sort<BigPiece, CF::THREADS>(L.pc, npc, (BigPiece*)&T0, l);
    big_rank_sort<BigRange, CF::THREADS>(L.rg, nrg, (BigRange*)&T0, l);
    __syncthreads();
  }
  const BigBlk* T = blk + s_base;
  if (bad) nb = 0;
  // emit staging in the U0 tile's LDS (free now): block-table entries, the splice's per-range words, the copy list
  BigGrp* const G = (BigGrp*)&T0;
  uint32_t* const dsx = (uint32_t*)((uint8_t*)&T0 + CF::SBG);
  if (!bad && DP.fast) big_ds_plan(dsv, dsp, eidx, DP, L.rg, nrg, dsx, (uint32_t)CF::MAXD);
  DIAGL(2);
  // ---- emit: pass 0 sizes (and proves the class), pass 1 bytes.  Every lane runs the same plan.
  uint64_t nblocks = 0, ndsc = 0, size = 0;
  const uint32_t ds0s = (uint32_t)s_ds0;
  uint32_t ngr = 0;
  uint64_t sbytes = 0;
  bool par = false;                                          // the parallel struct emit (planned in pass 0)
  for (int pass = 0; pass < 2 && !bad; pass++) {
    BigOut o; o.o = out + (pass ? s_at : 0); o.n = 0; o.w = pass == 1;
    // the copy list lives in the U0 tile's LDS past the block-table staging / client groups and the splice words
    o.cl = (BigCp*)(dsx + 3 * CF::MAXD); o.nc = 0; o.pre = s_cpre;
    o.cap = (uint32_t)((sizeof(typename CF::Tile) - CF::SBG - 12 * CF::MAXD) / sizeof(BigCp)); o.ls = o.le = o.ld = 0;
    o.cmd = &s_cmd; o.nw = CF::WAVES;
    if (L.patch) { o.pbits = S.pbits + PK.pb / 32u; o.pu0 = u0p; o.pn0 = n0; }   // (U0 structs whose info byte loses bit 0x20)
    o.vu(nblocks);
    if (pass == 0 && acanon) {
      uint64_t nbo = 0;
      const int pr = big_plan_structs(L, G, CF::GCAP, T, (uint32_t)nb, npc, S0, ds0s, ngr, nbo, sbytes);
      if (pr == 1) { bad = true; break; }
      par = pr == 0;
      if (par) nblocks = nbo;
    }
    if (par) {
      if (pass) big_write_structs(L, G, ngr, npc, u0p, arena, S0, ds0s, sbytes, o.n, o);
      o.n += sbytes;
    } else {
    uint64_t i = 0, nbo = 0;
    uint32_t j = 0;
    // U0 blocks no log piece touches (and whose headers are minimal) are U0's bytes [h0, b1) as
    // written: consecutive ones go out as one verbatim run [r0, r1)
    uint64_t r0 = 0, r1 = 0;
    // the block table is read through LDS (the U0 tile is free now): CF::SBN entries per refill
    uint64_t sc = ~0ull;
    const BigBlk* SB = (const BigBlk*)&T0;
    while ((i < nb || j < npc) && !bad) {
      if (i < nb && (sc == ~0ull || i >= sc + CF::SBN)) {
        const uint64_t m = nb - i < CF::SBN ? nb - i : CF::SBN;
        const uint4* g = (const uint4*)(T + i);
        uint4* t = (uint4*)&T0;
        wave_sync();
        for (uint32_t u = l; u < (uint32_t)m * (sizeof(BigBlk) / 16); u += WAVE) t[u] = g[u];
        wave_sync();
        sc = i;
      }
      if (i < nb) {
        // up to 64 untouched blocks at once: lane q tests block i + q (minimal header, client above the next
        // log piece's); the leading run of such blocks extends the verbatim run (U0 blocks are contiguous)
        const uint64_t cpx = j < npc ? 0xFFFFFFFFull - (L.pc[j].key >> 32) : 0;
        const uint64_t q = i + l;
        bool ok = q < nb && q < sc + CF::SBN;
        uint32_t h0q = 0, b1q = 0;
        if (ok) { const BigBlk& Q = SB[q - sc]; ok = Q.hcanon && (j >= npc || Q.client > cpx); h0q = Q.h0; b1q = Q.b1; }
        const uint64_t m = __ballot(ok);
        const uint32_t len = m == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~m);
        if (len) {
          const uint32_t h0 = (uint32_t)__builtin_amdgcn_readlane((int)h0q, 0);
          const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)b1q, (int)len - 1);
          if (r1 != h0) { if (r1 > r0) o.copy(u0p + r0, r1 - r0); r0 = h0; }
          r1 = b1; nbo += len; i += len;
          continue;
        }
      }
      const uint64_t cu = i < nb ? SB[i - sc].client : 0, cp = j < npc ? 0xFFFFFFFFull - (L.pc[j].key >> 32) : 0;
      const bool hu = i < nb && (j >= npc || cu >= cp);
      const uint64_t X = hu ? cu : cp;
      BigBlk B; if (hu) B = SB[i - sc];
      uint32_t j1 = j;
      while (j1 < npc && 0xFFFFFFFFull - (L.pc[j1].key >> 32) == X) j1++;
      if (hu && j1 == j && B.hcanon) {
        if (r1 != B.h0) { if (r1 > r0) o.copy(u0p + r0, r1 - r0); r0 = B.h0; }
        r1 = B.b1; nbo++; i++;
        continue;
      }
      if (r1 > r0) o.copy(u0p + r0, r1 - r0);
      r0 = r1 = 0;
      // items in clock order: the U0 block slots in before the first piece at or after its clock
      for (int sweep = 0; sweep < 2 && !bad; sweep++) {
        uint64_t cnt = 0, first = 0, pend = 0; bool any = false, pgc = false, upend = hu;
        uint32_t q = j;
        while (upend || q < j1) {
          const bool takeu = upend && (q >= j1 || B.clock0 <= (uint32_t)L.pc[q].key);
          const uint64_t c0 = takeu ? B.clock0 : (uint32_t)L.pc[q].key;
          const uint64_t c1 = takeu ? B.clock1 : c0 + L.pc[q].len;
          const bool fgc = takeu ? (bool)B.first_gc : L.pc[q].gc(), lgc = takeu ? (bool)B.last_gc : L.pc[q].gc();
          if (any) {
            if (c0 < pend || (c0 == pend && pgc && fgc)) { bad = true; break; }   // overlap / GC junction
            if (c0 > pend) { cnt++; if (sweep) { o.b(10); o.vu(c0 - pend); } }   // Skip over the gap
          } else first = c0;
          if (sweep) {
            if (takeu) o.copy(u0p + B.b0, B.b1 - B.b0);
            else o.copy(arena + L.pc[q].src, L.pc[q].nb());
          }
          cnt += takeu ? B.nst : 1u;
          any = true; pend = c1; pgc = lgc;
          if (takeu) upend = false; else q++;
        }
        if (sweep == 0 && !bad) { o.vu(cnt); o.vu(X); o.vu(first); }
      }
      nbo++;
      if (hu) i++;
      j = j1;
    }
    if (r1 > r0) o.copy(u0p + r0, r1 - r0);
    if (pass == 0) nblocks = nbo;
    }
    // delete set: U0's sorted stream (read through LDS tiles, forward only) merged with the sorted log
    // ranges, runs merged per client in one sweep.  Pass 0 keeps each client's run count in the struct
    // records' scratch (free after the clock-range pass) for pass 1's header.
#ifdef YGM_DIAG_BIGDS
    DIAG_PUT(6 + pass, __builtin_amdgcn_s_memrealtime());   // diagnostic: where the delete-set part of the pass starts
#endif
    uint64_t nc = 0;
    if (DP.fast) {
      // spliced: U0's entries no log range names are copied as written; a touched entry is its client, its new
      // run count, then its untouched ranges' bytes as written interleaved with the merged groups' spans
      const uint8_t* const dsb = u0p + s_ds0;
      const uint32_t ne = DP.C;
      o.vu(ndsc);
      // the parallel emit (its words: pass 0 in the empty copy list, pass 1 in the client-group region, whose struct
      // part is written by then; the same capacity both passes)
      const uint32_t wcap = (uint32_t)(CF::SBG / 4u) < o.cap * 4u ? (uint32_t)(CF::SBG / 4u) : o.cap * 4u;
      const bool dsdone = big_ds_par(L, DP, dsx, (uint32_t)CF::MAXD, nrg, pass ? (uint32_t*)G : (uint32_t*)o.cl, wcap, dsb, o, nc);
      uint32_t e = dsdone ? ne : 0u, r = dsdone ? nrg : 0u, cur = DP.b0;   // cur: byte start of entry e
      while (e < ne || r < nrg) {
        // U0's entries before the next log client's (big_ds_plan's lower bound) go out as one verbatim run
        const uint32_t e2 = r < nrg ? (L.rg[r].ent & 0x7FFFFFFFu) : ne;
        if (e < e2) {
          const uint32_t be = r < nrg ? dsx[r] : DP.bend;
          o.copy(dsb + cur, be - cur);
          nc += e2 - e; e = e2; cur = be;
          continue;
        }
        nc++;
        const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(L.rg[r].key >> 32);
        const bool touched = !(L.rg[r].ent >> 31);   // (then its entry is e)
        uint32_t cu = 0, n = 0, bs = 0, be = 0;
        if (touched) { cu = cl; n = dsx[CF::MAXD + r]; bs = cur; be = dsx[2 * CF::MAXD + r]; cur = be; }
        uint32_t r1 = r;
        while (r1 < nrg && (L.rg[r1].key >> 32) == (L.rg[r].key >> 32)) r1++;
        // groups of the client's log ranges (each widened by the U0 ranges it merges with): count, then write
        for (int sw = 0; sw < 2; sw++) {
          uint32_t ng = 0, cov = 0, gs = 0, ge = 0, ga = 0, gb = 0, gpa = 0, gpb = 0;
          uint32_t next = touched ? bs + vu_len(cu) + vu_len(n) : 0u;   // bytes of the next untouched U0 range
          bool have = false;
          auto close = [&]() __attribute__((always_inline)) {
            ng++; cov += gb - ga;
            if (sw) {
              if (touched && gpa > next) o.copy(dsb + next, gpa - next);
              o.vu(gs); o.vu(ge - gs);
              if (touched) next = gpb;
            }
          };
          for (uint32_t q = r; q < r1; q++) {
            const BigRange& R = L.rg[q];
            if (have && R.s <= ge) { if (R.e > ge) ge = R.e; if (R.b1 > gb) { gb = R.b1; gpb = R.pb; } }
            else { if (have) close(); gs = R.s; ge = R.e; ga = R.a; gb = R.b1; gpa = R.pa; gpb = R.pb; have = true; }
          }
          if (have) close();
          if (sw == 0) { o.vu(cl); o.vu(n - cov + ng); }
          else if (touched && be > next) o.copy(dsb + next, be - next);
        }
        if (touched) e++;
        r = r1;
      }
    } else {
    uint32_t* runs_of = dsv + dsn;
    const uint64_t runs_cap = ncap * (sizeof(BigRec) / 4) - dsn;
    BigDs D;
    D.s.init(dsv, dsn);
    uint64_t dprev = 0;
    auto dnext = [&]() __attribute__((always_inline)) {
      D.next();
      // U0's delete set in union order, every range inside 32-bit clocks (else the general path)
      if (D.has) { bad |= D.key < dprev || D.key + D.len > ((D.key >> 32) << 32) + 0xFFFFFFFFull; dprev = D.key; }
    };
    D.cl_left = D.s.next(); D.r_left = 0; D.client = 0;
    dnext();
    uint32_t r = 0;
    o.vu(ndsc);
    while ((D.has || r < nrg) && !bad) {
      const uint64_t kx = (D.has && (r >= nrg || D.key <= L.rg[r].key)) ? D.key : L.rg[r].key;
      const uint64_t hi = kx >> 32;
      if (pass) { o.vu(0xFFFFFFFFull - hi); o.vu(runs_of[nc]); }
      uint64_t runs = 0, rs = 0, re = 0;
      bool open = false;
      for (;;) {
        const bool du = D.has && (D.key >> 32) == hi, dl = r < nrg && (L.rg[r].key >> 32) == hi;
        if (!du && !dl) break;
        const bool tu = du && (!dl || D.key <= L.rg[r].key);
        const uint64_t ck = (uint32_t)(tu ? D.key : L.rg[r].key), ln = tu ? D.len : L.rg[r].len;
        if (open && ck <= re) { if (ck + ln > re) re = ck + ln; }
        else { if (open) { o.vu(rs); o.vu(re - rs); runs++; } rs = ck; re = ck + ln; open = true; }
        if (tu) dnext(); else r++;
      }
      if (open) { o.vu(rs); o.vu(re - rs); runs++; }
      if (!pass) {
        o.n += vu_len(0xFFFFFFFFull - hi) + vu_len(runs);
        if (nc >= runs_cap) bad = true;
        else if (l == 0) runs_of[nc] = (uint32_t)runs;
      }
      nc++;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // pass 0's run counts before pass 1 reads them
    bad |= D.s.err;
    }
    o.flush();
    DIAGL(3 + pass);
    if (pass == 0) {
      ndsc = nc; size = o.n;
      bad |= ((flags & 1u) && nc > 1) ;                       // yjs 13.5: first-seen client order -> general path
      // the header varuints were sized with 0: resize with the real counts
      size += vu_len(nblocks) - 1 + vu_len(ndsc) - 1;
      if (!bad && l == 0) {
        const uint64_t at = merge_place(upd_off, doc_upd, d, size, slot_total, meta);
        s_at = at;
        if (at + size > out_cap) L.bad = 1;
      }
      wave_sync();
      bad |= L.bad != 0;
    }
  }
  if (l == 0) s_cmd.cmd = 0;   // the helper waves leave
  __syncthreads();
  if (l == 0) {
    if (bad) { status[d] = ST_FALLBACK; fb2_list[atomicAdd(&meta->big_defer, 1u)] = d; }
    else { out_off[d] = s_at; out_len[d] = size; status[d] = ST_OK; add_payload(meta, d, size); }
  }
}

// ======================================================================= merge sequential
// One lane per fallback document.  Scratch (readers, sort arrays, block
// counts, delete-set records) is carved with atomic cursors.
struct SeqScratch {
  Stream* readers; int* order; int* tmp; const uint8_t** ubase; uint32_t* ulen;  // per update
  uint32_t* cnt; DRec* drec;                                                       // per input byte
  uint64_t upd_cap, byte_cap;
};

__global__ __launch_bounds__(64) void k_merge_seq(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                  const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ fb_list,
                                                  uint32_t n_fb, uint32_t flags, uint8_t* __restrict__ out,
                                                  uint64_t* __restrict__ out_off, uint64_t* __restrict__ out_len,
                                                  int32_t* __restrict__ status, DocMeta* meta, SeqScratch scr, uint64_t slot_total,
                                                  uint64_t out_cap) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_fb) return;
  const uint32_t d = fb_list[q];
  const uint32_t u0 = doc_upd[d], u1 = doc_upd[d + 1];
  const int k = (int)(u1 - u0);
  const uint64_t b0 = upd_off[u0], b1 = upd_off[u1];
  const uint64_t nbytes = b1 - b0;
  const uint64_t su = atomicAdd(&meta->scr_upd_cursor, (unsigned long long)k);
  const uint64_t sb = atomicAdd(&meta->scr_byte_cursor, (unsigned long long)(nbytes + 8));
  int st = ST_OK;
  if (su + k > scr.upd_cap || sb + nbytes + 8 > scr.byte_cap) st = ST_NOMEM;
  Stream* R = scr.readers + su; int* order = scr.order + su; int* tmp = scr.tmp + su;
  const uint8_t** ub = scr.ubase + su; uint32_t* ul = scr.ulen + su;
  uint32_t* cnt = scr.cnt + sb;
  DRec* drec = scr.drec + (sb / 2);  // DS records need <= nbytes/3 entries of 40 B: carved from a 20x-byte region
  const uint64_t cnt_cap = nbytes + 8, drec_cap = (nbytes + 8) / 2;
  uint64_t size = 0, nblocks = 0;
  if (st == ST_OK) {
    for (int i = 0; i < k; i++) { const uint64_t a = upd_off[u0 + i], b = upd_off[u0 + i + 1]; ub[i] = arena + a; ul[i] = (uint32_t)(b - a); }
    Out o{nullptr, 0};
    LW lw{&o, false, flags, 0, 0, 0, cnt, cnt_cap, 0, false};
    st = merge_pass(R, order, tmp, k, ub, ul, flags, lw);
    if (st == ST_OK) {
      nblocks = lw.bi;
      o.vu(nblocks);
      const int64_t nr = ds_collect(R, k, drec, drec_cap);
      if (nr < 0) st = (int)(-nr);
      else if (lw.nc) st = ST_NONCANON;
      else { ds_union_write(drec, (uint64_t)nr, flags, o); size = o.n; }
    }
  }
  uint64_t at = 0;
  if (st == ST_OK) {
    at = merge_place(upd_off, doc_upd, d, size, slot_total, meta);
    if (at + size > out_cap) st = ST_NOMEM;
  }
  if (st == ST_OK) {  // write pass: block count, structs, delete set
    Out o{out + at, 0};
    o.vu(nblocks);
    LW lw{&o, true, flags, 0, 0, 0, cnt, cnt_cap, 0, false};
    st = merge_pass(R, order, tmp, k, ub, ul, flags, lw);
    if (st == ST_OK) {
      const int64_t nr = ds_collect(R, k, drec, drec_cap);
      if (nr < 0) st = (int)(-nr);
      else ds_union_write(drec, (uint64_t)nr, flags, o);
    }
  }
  if (st == ST_OK) add_payload(meta, d, size);
  out_off[d] = at; out_len[d] = st == ST_OK ? size : 0; status[d] = st;
}

}  // namespace ygm

// ======================================================================= launch glue (helpers: ygm_docmeta.hpp)
extern "C" {

using namespace ygm;

#ifdef YGM_DIAG
int ygm_diag_ts_read(unsigned long long* out, int reset) {  // 16384 x 8 stamps of the lean kernel
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ygm_diag_ts), sizeof(unsigned long long) * 16384 * 8) != hipSuccess) return -1;
  (void)reset;
  return 0;
}
int ygm_diag_ds_read(unsigned long long* out, int reset) {   // 4 delete-set union cycle sums
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ygm_diag_ds), sizeof(unsigned long long) * 4) != hipSuccess) return -1;
  if (reset) { unsigned long long z[4] = {0}; (void)hipMemcpyToSymbol(HIP_SYMBOL(ygm_diag_ds), z, sizeof z); }
  return 0;
}
int ygm_diag_read(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ygm_diag), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
  if (reset) { unsigned long long z[32] = {0}; (void)hipMemcpyToSymbol(HIP_SYMBOL(ygm_diag), z, sizeof z); }
  return 0;
}
#endif

size_t ygm_k_big_blk_bytes() { return sizeof(BigBlk); }
size_t ygm_k_big_rec_bytes() { return sizeof(BigRec); }
// the snapshot scan's scratch for n_fb large documents of fb_bytes in all: counters, picks, tasks, nx, vl
static void big_scan_layout(uint32_t n_fb, uint64_t fb_bytes, BigScan& S, uint8_t* base, size_t& total) {
  S.ntask_cap = fb_bytes / BIG_SCAN_CH + n_fb + 1;
  S.npos_cap = fb_bytes + 48ull * n_fb + 16;
  S.vq_cap = S.npos_cap / 4 + 1024;
  size_t o = 0;
  auto carve = [&](size_t bytes) { const size_t a = o; o += (bytes + 255) & ~(size_t)255; return base ? base + a : nullptr; };
  S.cnt = (unsigned long long*)carve(64);
  S.pick = (BigPick*)carve(sizeof(BigPick) * (size_t)n_fb);
  S.task = (uint2*)carve(sizeof(uint2) * S.ntask_cap);
  S.nv = (uint32_t*)carve(4 * S.npos_cap);
  S.llist = (uint32_t*)carve(4ull * n_fb);
  S.mlist = (uint32_t*)carve(4ull * n_fb);
  S.vq = (uint2*)carve(sizeof(uint2) * S.vq_cap);
  S.pbits = (uint32_t*)carve(4 * (S.npos_cap / 32 + 4));
  total = o;
}
// device pointers of the scan's counters and of its two document lists (after ygm_k_launch_big_scan)
void ygm_k_big_lists(void* scan, uint32_t n_fb, uint64_t fb_bytes, unsigned long long** cnt, uint32_t** llist, uint32_t** mlist) {
  BigScan S; size_t total;
  big_scan_layout(n_fb, fb_bytes, S, (uint8_t*)scan, total);
  *cnt = S.cnt; *llist = S.llist; *mlist = S.mlist;
}
size_t ygm_k_big_scan_bytes(uint32_t n_fb, uint64_t fb_bytes) { BigScan S; size_t t; big_scan_layout(n_fb, fb_bytes, S, nullptr, t); return t; }
int ygm_k_launch_big_scan(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list,
                          uint32_t n_fb, uint32_t flags, void* scan, uint64_t fb_bytes, hipStream_t s) {
  if (n_fb == 0) return 0;
  BigScan S; size_t total;
  big_scan_layout(n_fb, fb_bytes, S, (uint8_t*)scan, total);
  if (hipMemsetAsync(S.cnt, 0, 64, s) != hipSuccess) return launch_rc(__func__);
  hipLaunchKernelGGL(k_big_pick, dim3((n_fb + 15) / 16), dim3(1024), 0, s, arena, upd_off, doc_upd, fb_list, n_fb, S);
  // the scan: a persistent grid over the tasks (at most 16 workgroups per CU; the task count is on the device)
  const uint64_t g = S.ntask_cap < 16ull * device_cus() ? S.ntask_cap : 16ull * device_cus();
  hipLaunchKernelGGL(k_big_scan, dim3((uint32_t)g), dim3(256), 0, s, arena, upd_off, doc_upd, fb_list, flags, S);
  const uint64_t gv = S.vq_cap / 256 + 1 < 8ull * device_cus() ? S.vq_cap / 256 + 1 : 8ull * device_cus();
  hipLaunchKernelGGL(k_big_val, dim3((uint32_t)gv), dim3(256), 0, s, arena, upd_off, doc_upd, fb_list, flags, S);
  return launch_rc(__func__);
}
// The mid size starts after the 16-wave size's workgroups are resident: a 16-wave workgroup needs a whole CU (its LDS),
// and once the mid size's four-per-CU workgroups (tens of thousands queued behind them) hold every CU, no CU drains
// whole until the mid size is nearly done -- the 16-wave documents then start late, and the batch takes their whole
// time after the mid size's (C3: 35 -> 50 ms on such runs).  One wave on the mid size's stream waits for the count
// the 16-wave workgroups raise as they start, for at most 1 ms: s_memrealtime is the 100 MHz constant clock
// (s_memtime counts shader cycles, whose rate follows the clock governor), 100 000 ticks.  The bound matters when the
// second stream shares a hardware queue with the first (a process with more streams than queues): the 16-wave kernel
// then queues behind the mid size and cannot start, and the wait costs its whole 1 ms.
__global__ __launch_bounds__(64) void k_big_wait(DocMeta* meta, uint32_t want) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(&meta->big_started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want &&
         __builtin_amdgcn_s_memrealtime() - t0 < 100000ull)
    __builtin_amdgcn_s_sleep(8);
}
int ygm_k_launch_big_wait(void* meta, uint32_t n_large, hipStream_t s) {
  const uint32_t ncu = device_cus();
  const uint32_t want = n_large < ncu ? n_large : ncu;
  if (want == 0) return 0;
  hipLaunchKernelGGL(k_big_wait, dim3(1), dim3(64), 0, s, (DocMeta*)meta, want);
  return launch_rc(__func__);
}
// large = 0: the mid size, large = 1: the 16-wave size, over the fb_list indices in fbx[0, n) (the mid size sends a
// document whose log exceeds its LDS to up_list, meta->mid_defer)
int ygm_k_launch_merge_big(int large, const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list,
                           uint32_t n_fb, const uint32_t* fbx, uint32_t n, uint32_t* up_list, uint32_t flags, uint8_t* out,
                           uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta, uint32_t* fb2_list, void* blk,
                           uint64_t blk_cap, void* rec, uint64_t rec_cap, uint64_t slot_total, uint64_t out_cap, void* scan,
                           uint64_t fb_bytes, hipStream_t s) {
  if (n == 0) return 0;
  BigScan S; size_t total;
  big_scan_layout(n_fb, fb_bytes, S, (uint8_t*)scan, total);
  if (large)
    hipLaunchKernelGGL(k_merge_big<BigCfgL>, dim3(n), dim3(BigCfgL::THREADS), 0, s, arena, upd_off, doc_upd, fb_list, flags, out, out_off,
                       out_len, status, (DocMeta*)meta, fb2_list, (BigBlk*)blk, blk_cap, (BigRec*)rec, rec_cap, slot_total, out_cap, S,
                       fbx, up_list);
  else
    hipLaunchKernelGGL(k_merge_big<BigCfgM>, dim3(n), dim3(BigCfgM::THREADS), 0, s, arena, upd_off, doc_upd, fb_list, flags, out, out_off,
                       out_len, status, (DocMeta*)meta, fb2_list, (BigBlk*)blk, blk_cap, (BigRec*)rec, rec_cap, slot_total, out_cap, S,
                       fbx, up_list);
  return launch_rc(__func__);
}
size_t ygm_k_meta_bytes() { return sizeof(DocMeta); }
int ygm_k_meta_layout(size_t* sz, size_t* off_big_started, size_t* off_big_scur, size_t* off_payload_sh) {
  *sz = sizeof(DocMeta); *off_big_started = offsetof(DocMeta, big_started); *off_big_scur = offsetof(DocMeta, big_scur);
  *off_payload_sh = offsetof(DocMeta, payload_sh);
  return 0;
}
size_t ygm_k_seq_reader_bytes() { return sizeof(Stream); }
size_t ygm_k_drec_bytes() { return sizeof(DRec); }

int ygm_k_launch_doc(int mode, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                     const uint32_t* docs, uint64_t out_base, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                     uint64_t* out_len, int32_t* status, unsigned long long* lb, void* meta, uint64_t out_cap, hipStream_t s) {
  const uint32_t tiles = (n_docs + DOC_NT - 1) / DOC_NT;
  if (tiles == 0) return 0;
  if (mode == 0)
    hipLaunchKernelGGL(k_doc<0>, dim3(tiles), dim3(DOC_NT), 0, s, arena, doc_off, sv_arena, sv_off, docs, out_base, n_docs, flags, out, out_off, out_len, status, lb, (DocMeta*)meta, out_cap);
  else
    hipLaunchKernelGGL(k_doc<1>, dim3(tiles), dim3(DOC_NT), 0, s, arena, doc_off, sv_arena, sv_off, docs, out_base, n_docs, flags, out, out_off, out_len, status, lb, (DocMeta*)meta, out_cap);
  return launch_rc(__func__);
}

// ======================================================================= host API: packed results
// The device results leave each document's bytes in its own slot; the host API copies back only the
// outputs, packed in document order: per-256-document sums, one scan of those sums, each document's packed offset,
// then the copy by 16 KB chunks of the packed output (16-byte pieces, byte stores for a segment's last partial piece:
// the chunks' byte ranges are disjoint).
__global__ __launch_bounds__(DOC_NT) void k_pack_sum(const uint64_t* __restrict__ len, const int32_t* __restrict__ status, uint32_t n,
                                                   uint64_t* __restrict__ bsum) {
  __shared__ uint64_t tmp[DOC_NT / WAVE + 1];
  const uint32_t d = blockIdx.x * DOC_NT + threadIdx.x;
  const uint64_t v = d < n && status[d] == ST_OK ? len[d] : 0ull;
  uint64_t tot;
  (void)block_exscan<DOC_NT>(v, tmp, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(1024) void k_pack_scan(uint64_t* __restrict__ bsum, uint32_t nb) {
  __shared__ uint64_t tmp[1024 / WAVE + 1];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint32_t i = b0 + threadIdx.x;
    const uint64_t v = i < nb ? bsum[i] : 0ull;
    uint64_t tot;
    const uint64_t pre = block_exscan<1024>(v, tmp, tot);
    if (i < nb) bsum[i] = carry + pre;
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}
__global__ __launch_bounds__(DOC_NT) void k_pack_off(const uint64_t* __restrict__ len, const int32_t* __restrict__ status, uint32_t n,
                                                   const uint64_t* __restrict__ bsum, uint64_t* __restrict__ poff) {
  __shared__ uint64_t tmp[DOC_NT / WAVE + 1];
  const uint32_t d = blockIdx.x * DOC_NT + threadIdx.x;
  const uint64_t v = d < n && status[d] == ST_OK ? len[d] : 0ull;
  uint64_t tot;
  const uint64_t at = bsum[blockIdx.x] + block_exscan<DOC_NT>(v, tmp, tot);
  if (d < n) poff[d] = at;
}
// the copy: a wave per 16 KB chunk of the packed output (persistent grid; the total from the scan), so that a document
// of megabytes is copied by as many waves as it has chunks (a wave per document left one wave copying C3's 10 MB
// document, and C5's 380 KB documents 64 to a wave: 10-20 ms).  The chunk's first document by a 64-way search of the
// offsets (one load per lane and step), then the documents it spans, 16-byte pieces per lane.
constexpr uint64_t PK_CH = 16384;
__global__ __launch_bounds__(256) void k_pack_chunks(const uint8_t* __restrict__ src, const uint64_t* __restrict__ off, uint32_t n,
                                                     const uint64_t* __restrict__ poff, const uint64_t* __restrict__ total_p,
                                                     uint8_t* __restrict__ dst) {
  const uint32_t l = threadIdx.x % WAVE;
  const uint64_t total = *total_p, nch = (total + PK_CH - 1) / PK_CH;
  const uint64_t W = (uint64_t)gridDim.x * (256 / WAVE);
  for (uint64_t c = (uint64_t)blockIdx.x * (256 / WAVE) + threadIdx.x / WAVE; c < nch; c += W) {
    const uint64_t s = c * PK_CH, e = s + PK_CH < total ? s + PK_CH : total;
    // the last document d with poff[d] <= s (poff nondecreasing, poff[0] = 0)
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1u) {
      const uint32_t step = (hi - lo + WAVE - 1u) / WAVE, i = lo + l * step;
      const bool le = i < hi && poff[i] <= s;
      const uint64_t m = __ballot(le);   // (a prefix of the lanes; lane 0 holds: poff[lo] <= s)
      const uint32_t k = 63u - (uint32_t)__builtin_clzll(m);
      lo += k * step;
      hi = lo + step < hi ? lo + step : hi;
    }
    for (uint32_t d = lo; d < n; d++) {
      const uint64_t a = poff[d];
      if (a >= e) break;
      const uint64_t b = d + 1u < n ? poff[d + 1u] : total;
      const uint64_t x0 = a > s ? a : s, x1 = b < e ? b : e;
      const uint8_t* sp = src + off[d] + (x0 - a);
      uint8_t* dp = dst + x0;
      const uint64_t L = x1 > x0 ? x1 - x0 : 0ull;
      for (uint64_t q = 16ull * l; q < L; q += 16ull * WAVE) {
        if (q + 16 <= L) { u32x4 x; __builtin_memcpy(&x, sp + q, 16); __builtin_memcpy(dp + q, &x, 16); }
        else for (uint64_t k = q; k < L; k++) dp[k] = sp[k];
      }
    }
  }
}
int ygm_k_launch_pack(const uint8_t* src, const uint64_t* off, const uint64_t* len, const int32_t* status, uint32_t n, uint64_t* bsum,
                      uint8_t* dst, uint64_t* poff, hipStream_t s) {
  if (n == 0) return 0;
  const uint32_t nb = (n + DOC_NT - 1) / DOC_NT;
  hipLaunchKernelGGL(k_pack_sum, dim3(nb), dim3(DOC_NT), 0, s, len, status, n, bsum);
  hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(1024), 0, s, bsum, nb);
  hipLaunchKernelGGL(k_pack_off, dim3(nb), dim3(DOC_NT), 0, s, len, status, n, (const uint64_t*)bsum, poff);
  hipLaunchKernelGGL(k_pack_chunks, dim3(8u * device_cus()), dim3(256), 0, s, src, off, n, (const uint64_t*)poff,
                     (const uint64_t*)(bsum + nb), dst);
  return launch_rc(__func__);
}

// workgroups of `threads` resident at once on the device (occupancy x CUs), for persistent grids
extern "C++" template <class K>
static uint32_t resident_blocks(K kernel, int threads, uint32_t fallback) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess || cus <= 0 || per <= 0)
    return fallback;
  return (uint32_t)(cus * per);
}

uint32_t ygm_k_lean_stage_bytes() { return (uint32_t)LN_IN; }   // input bytes the narrow lean kernel stages per document
// doc_off / upd_len non-null: the compact input form (ygm_merge_v1_device_lens); upd_off is then unused
int ygm_k_launch_merge_lean(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, uint32_t flags,
                            uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta, void* meta_next,
                            uint32_t* defer_list, uint64_t out_cap, hipStream_t s, const uint64_t* doc_off, const uint16_t* upd_len) {
  if (n_docs == 0) return 0;
  // persistent waves: enough for full occupancy, each looping over documents d, d + G, ...
  const int n_cu = (int)device_cus();
  const char* env = getenv("YGM_LEAN_WAVES_PER_CU");
  const uint32_t wpc = env ? (uint32_t)atoi(env) : 16u;
  const uint32_t grid = n_docs < (uint32_t)n_cu * wpc ? n_docs : (uint32_t)n_cu * wpc;
  if (doc_off)
    hipLaunchKernelGGL((k_merge_lean<0, 1>), dim3(grid), dim3(WAVE), 0, s, arena, upd_off, doc_upd, n_docs, flags, out, out_off, out_len,
                       status, (DocMeta*)meta, (DocMeta*)meta_next, defer_list, out_cap, (const uint32_t*)nullptr, 0u, doc_off, upd_len);
  else
    hipLaunchKernelGGL((k_merge_lean<0, 0>), dim3(grid), dim3(WAVE), 0, s, arena, upd_off, doc_upd, n_docs, flags, out, out_off, out_len,
                       status, (DocMeta*)meta, (DocMeta*)meta_next, defer_list, out_cap, (const uint32_t*)nullptr, 0u,
                       (const uint64_t*)nullptr, (const uint16_t*)nullptr);
  return launch_rc(__func__);
}
// The update-offset table of the compact input form, for the documents of `list` (every document: list == nullptr):
// a wave per document scans its lengths from its base.  An offset past the document's end is clamped to it (lengths
// that do not add up to the document: its updates then fail to parse -- an error status, never a read outside it).
__global__ __launch_bounds__(256) void k_build_off(const uint64_t* __restrict__ doc_off, const uint16_t* __restrict__ upd_len,
                                                   const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ list, uint32_t n,
                                                   uint64_t* __restrict__ upd_off) {
  const uint32_t w = blockIdx.x * 4u + threadIdx.x / WAVE, l = threadIdx.x % WAVE;
  if (w >= n) return;
  const uint32_t d = list ? list[w] : w;
  const uint32_t u0 = doc_upd[d], u1 = doc_upd[d + 1];
  const uint64_t b0 = doc_off[d], b1 = doc_off[d + 1];
  uint64_t carry = b0;
  for (uint32_t c = u0; c < u1; c += WAVE) {
    const uint32_t i = c + l;
    const uint32_t len = i < u1 ? upd_len[i] : 0u;
    const uint32_t inc = dpp_incl_add(len);
    const uint64_t off = carry + inc - len;
    if (i < u1) upd_off[i] = off < b1 ? off : b1;
    carry += lane63(inc);
  }
  // lengths that do not add up to the document (include/ygm.h: an error status): with two or more updates every
  // one becomes empty, which no tier parses (yjs: readVarUint past the end throws); a single update is checked
  // where it is passed through (the lean kernels' single path reads upd_len)
  if (carry != b1 && u1 - u0 >= 2u)
    for (uint32_t i = u0 + l; i < u1; i += WAVE) upd_off[i] = b1;
  if (l == 0) upd_off[u1] = b1;
}
int ygm_k_launch_build_off(const uint64_t* doc_off, const uint16_t* upd_len, const uint32_t* doc_upd, const uint32_t* list, uint32_t n,
                           uint64_t* upd_off, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_build_off, dim3((n + 3) / 4), dim3(256), 0, s, doc_off, upd_len, doc_upd, list, n, upd_off);
  return launch_rc(__func__);
}
// the wide lean kernel over the narrow one's deferred list (n_list entries); its own deferrals go to defer_list
// (count: DocMeta::wide_defer)
int ygm_k_launch_merge_lean_wide(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, const uint32_t* list,
                                 uint32_t n_list, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status,
                                 void* meta, void* meta_next, uint32_t* defer_list, uint64_t out_cap, const uint16_t* upd_len, hipStream_t s) {
  if (n_list == 0) return 0;
  static std::atomic<uint32_t> cache[YGM_MAX_DEVICES];
  const uint32_t resident = per_device(cache, [] { const char* g = getenv("YGM_WIDE_GRID"); return g ? (uint32_t)atoi(g) : resident_blocks(k_merge_lean<1, 0>, WAVE, 2048u); });
  const uint32_t grid = n_list < resident ? n_list : resident;
  hipLaunchKernelGGL((k_merge_lean<1, 0>), dim3(grid), dim3(WAVE), 0, s, arena, upd_off, doc_upd, n_docs, flags, out, out_off, out_len,
                     status, (DocMeta*)meta, (DocMeta*)meta_next, defer_list, out_cap, list, n_list, (const uint64_t*)nullptr,
                     upd_len);
  return launch_rc(__func__);
}

int ygm_k_launch_merge_wave(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs,
                            const unsigned int* n_dev, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                            int32_t* status, void* meta, uint32_t* defer_list, uint32_t* fb_list, uint64_t out_cap, hipStream_t s) {
  if (n_docs == 0) return 0;
  // persistent: exactly the waves that are resident at once (LDS / VGPR occupancy x CUs), so no wave starts
  // its grid-stride share after the others have finished theirs; n_docs is the upper bound of the device count
  static std::atomic<uint32_t> cache[YGM_MAX_DEVICES];
  const uint32_t resident = per_device(cache, [] { const char* g = getenv("YGM_WAVE_GRID"); return g ? (uint32_t)atoi(g) : resident_blocks(k_merge_wave, WAVE, 2048u); });
  const uint32_t grid = n_docs < resident ? n_docs : resident;
  hipLaunchKernelGGL(k_merge_wave, dim3(grid), dim3(WAVE), 0, s, arena, upd_off, doc_upd, docs, n_dev, n_docs,
                     flags, out, out_off, out_len, status, (DocMeta*)meta, defer_list, fb_list, out_cap);
  return launch_rc(__func__);
}

int ygm_k_launch_route_big(const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs, const unsigned int* n_dev, uint32_t n_docs,
                           uint32_t flags, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta, uint32_t* fb_list, uint32_t* rest,
                           hipStream_t s) {
  if (n_docs == 0) return 0;
  const uint32_t grid = (n_docs + 255u) / 256u < 2048u ? (n_docs + 255u) / 256u : 2048u;   // (n_docs: the bound of the device count)
  hipLaunchKernelGGL(k_route_big, dim3(grid), dim3(256), 0, s, upd_off, doc_upd, docs, n_dev, n_docs, flags, out_off, out_len, status,
                     (DocMeta*)meta, fb_list, rest);
  return launch_rc(__func__);
}

int ygm_k_launch_merge_fast(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs,
                            const unsigned int* n_dev, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                            int32_t* status, uint64_t slot_total, void* meta, uint32_t* fb_list, uint64_t out_cap, hipStream_t s) {
  if (n_docs == 0) return 0;
  static std::atomic<uint32_t> cache[YGM_MAX_DEVICES];   // persistent: the resident workgroups (see ygm_k_launch_merge_wave)
  const uint32_t resident = per_device(cache, [] { const char* g = getenv("YGM_FAST_GRID"); return g ? (uint32_t)atoi(g) : resident_blocks(k_merge_fast, M_NT, 512u); });
  const uint32_t grid = n_docs < resident ? n_docs : resident;
  hipLaunchKernelGGL(k_merge_fast, dim3(grid), dim3(M_NT), 0, s, arena, upd_off, doc_upd, docs, n_dev, n_docs, flags, out, out_off, out_len,
                     status, slot_total, (DocMeta*)meta, fb_list, out_cap);
  return launch_rc(__func__);
}

int ygm_k_launch_merge_seq(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list, uint32_t n_fb,
                           uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta,
                           void* readers, int* order, int* tmp, const uint8_t** ubase, uint32_t* ulen, uint64_t upd_cap,
                           uint32_t* cnt, void* drec, uint64_t byte_cap, uint64_t slot_total, uint64_t out_cap, hipStream_t s) {
  if (n_fb == 0) return 0;
  SeqScratch scr{(Stream*)readers, order, tmp, ubase, ulen, cnt, (DRec*)drec, upd_cap, byte_cap};
  hipLaunchKernelGGL(k_merge_seq, dim3((n_fb + 63) / 64), dim3(64), 0, s, arena, upd_off, doc_upd, fb_list, n_fb, flags, out, out_off,
                     out_len, status, (DocMeta*)meta, scr, slot_total, out_cap);
  return launch_rc(__func__);
}

}  // extern "C"
