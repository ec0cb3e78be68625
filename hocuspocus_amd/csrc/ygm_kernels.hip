// ygm_kernels.hip -- gfx950 kernels of the batched Yjs update engine.
//
//  k_sv          encodeStateVectorFromUpdate, one lane per document   (yjs Y@37728)
//  k_diff        diffUpdate, one lane per document                    (yjs Y@40711)
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

#include "ygm_common.hpp"
#include "ygm_merge_seq.hpp"
#include "ygm_merge_wave.hpp"
#include "ygm_seqdoc.hpp"
#include "ygm_v1.hpp"

#ifdef YGM_DIAG
// diagnostic build only (libygm_diag.so): per-phase shader-clock sums of k_merge_fast
__device__ unsigned long long ygm_diag[16];
#define DIAG_T0 unsigned long long _dt = __builtin_amdgcn_s_memtime();
#define DIAG(i) do { if (threadIdx.x == 0) { unsigned long long _n = __builtin_amdgcn_s_memtime(); atomicAdd(&ygm_diag[i], _n - _dt); _dt = _n; } } while (0)
#define DIAGW(i) do { if ((threadIdx.x & 63) == 0) { unsigned long long _n = __builtin_amdgcn_s_memtime(); atomicAdd(&ygm_diag[8 + (i)], _n - _dt); _dt = _n; } } while (0)
#else
#define DIAGW(i)
#define DIAG_T0
#define DIAG(i)
#endif

namespace ygm {

// ======================================================================= SV / diff
constexpr int DOC_NT = 256;   // lanes (= documents) per workgroup tile
constexpr int DIFF_BLK = 16;  // per-lane LDS slots for output-block counts

struct DocMeta {                    // per-launch device counters (zeroed by the launcher)
  unsigned int ticket;
  unsigned int fault;
  unsigned int fb_count;            // documents sent to the sequential kernel
  unsigned int defer_count;         // documents sent from the wave kernel to the workgroup kernel
  unsigned int ticket_m;            // tickets of the workgroup kernel
  unsigned int pad[3];
  unsigned long long fast_total;    // bytes in the first look-back region
  unsigned long long m_total;       // bytes in the workgroup-kernel region (after fast_total)
  unsigned long long seq_cursor;    // bytes appended by the sequential kernel
  unsigned long long fb_upds;       // updates / bytes of fallback documents (scratch sizing)
  unsigned long long fb_bytes;
  unsigned long long scr_upd_cursor;
  unsigned long long scr_byte_cursor;
};

template <int MODE>  // 0 = sv, 1 = diff
__global__ __launch_bounds__(DOC_NT) void k_doc(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off,
                                                 const uint8_t* __restrict__ sv_arena, const uint64_t* __restrict__ sv_off,
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
  const uint32_t d = tile * DOC_NT + threadIdx.x;
  const bool live = d < n_docs;
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
  const uint64_t at = s_base + pre;
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
      SInfo si; read_struct(c, si, flags);
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

// Documents deferred by the wave kernel (list `docs`, n_docs entries); output
// region starts at meta->fast_total.
__global__ __launch_bounds__(M_NT) void k_merge_fast(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                      const uint32_t* __restrict__ doc_upd, const uint32_t* __restrict__ docs,
                                                      uint32_t n_docs, uint32_t flags,
                                                      uint8_t* __restrict__ out_all, uint64_t* __restrict__ out_off,
                                                      uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                                                      unsigned long long* lb, DocMeta* meta, uint32_t* fb_list, uint64_t out_cap) {
  __shared__ MergeLds L;
  const int t = threadIdx.x;
  DIAG_T0
  if (t == 0) { L.tile = atomicAdd(&meta->ticket_m, 1u); L.err = 0; L.fb = 0; L.nc = 0; }
  __syncthreads();
  const uint32_t tile = L.tile;
  const uint32_t d = docs[tile];
  const uint64_t region = meta->fast_total;
  uint8_t* out = out_all + region;
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
      else if ((flags & F_COMPAT_135) && D > 0) st = ST_FALLBACK;  // first-seen DS order: sequential kernel
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
      const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(kj >> 32), ck = (uint32_t)kj;
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
  // ---- look-back: this document's place in the packed output
  const uint64_t mysz = (st == ST_OK) ? size : 0;
  if (t < WAVE) {
    const uint64_t b = lookback(lb, tile, mysz, &meta->fault);
    if (t == 0) {
      L.base = b;
      if (tile == n_docs - 1) meta->m_total = b + mysz;
      if (st == ST_FALLBACK) {
        const uint32_t q = atomicAdd(&meta->fb_count, 1u);
        fb_list[q] = d;
        atomicAdd(&meta->fb_upds, (unsigned long long)k);
        atomicAdd(&meta->fb_bytes, (unsigned long long)nbytes);
      }
    }
  }
  __syncthreads();
  DIAG(6);
  const uint64_t base = L.base;
  if (meta->fault && st == ST_OK) st = ST_DEVICE;
  if (st == ST_OK && region + base + size > out_cap) st = ST_NOMEM;
  if (t == 0) { out_off[d] = region + base; out_len[d] = st == ST_OK ? size : 0; status[d] = st == ST_FALLBACK ? ST_FALLBACK : st; }
  if (st != ST_OK) return;
  uint8_t* o = out + base;
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
      else { Cur c{L.in, L.r_start[r], L.ustart[L.r_src[r]] + L.ulen[L.r_src[r]], 0, 0}; SInfo si; read_struct(c, si, flags); write_struct(w, L.in, si, cl, ck, 0, false, flags); }
    }
  }
  // ---- emit delete set
  const uint32_t dsb = hdr0 + struct_bytes;
  if (t == 0) { Out w{o + dsb, 0}; w.vu(L.nseg); }
  const uint32_t dh = vu_len(L.nseg);
  for (int j = t; j < D; j += M_NT) {
    const uint32_t f = L.dF[j]; const uint64_t kj = L.dkey[j];
    const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(kj >> 32), ck = (uint32_t)kj;
    Out w{o + dsb + dh + (uint32_t)L.dA[j], 0};
    if (f & 1u) { w.vu(cl); w.vu(L.dC[L.dB[j]]); }
    if (f & 2u) { w.vu(ck); w.vu(L.dE[j] - ck); }
  }
  DIAG(7);
}


// ======================================================================= merge: one wave per document
// Per-element state lives in LDS (eflag/eblk/epos, dflag/dsid/dposs) and every
// per-element loop is rolled: the kernel stays small enough for the I-cache.
__global__ __launch_bounds__(WAVE * W_WAVES) void k_merge_wave(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off,
                                                               const uint32_t* __restrict__ doc_upd, uint32_t n_docs, uint32_t flags,
                                                               uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                                                               uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                                                               unsigned long long* lb, DocMeta* meta, uint32_t* defer_list,
                                                               uint32_t* fb_list, uint64_t out_cap) {
  __shared__ WaveLds LS[W_WAVES];
  DIAG_T0
  const uint32_t l = threadIdx.x % WAVE;
  WaveLds& L = LS[threadIdx.x / WAVE];
  uint32_t tk = 0;
  if (l == 0) tk = atomicAdd(&meta->ticket, 1u);
  const uint32_t d = (uint32_t)__shfl((int)tk, 0, WAVE);
  if (d >= n_docs) return;
  const uint32_t u0 = doc_upd[d], u1 = doc_upd[d + 1];
  const uint32_t k = u1 - u0;
  const uint64_t b0 = upd_off[u0], b1 = upd_off[u1];
  const uint64_t nbytes = b1 - b0;
  constexpr int ST_DEFER = 101;
  int st = ST_OK, mode = 0;
  uint64_t size = 0;
  uint32_t S = 0, D = 0, nblocks = 0, nseg = 0, hdr0 = 0, sbytes = 0, dsbytes = 0;
  if (k == 0) { mode = 1; size = 2; }
  else if (k == 1) { mode = 2; size = nbytes; }
  else if (k > (uint32_t)W_K || nbytes + 16 > (uint64_t)W_IN || (flags & 2u)) st = ST_DEFER;
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
    wave_sync();
    DIAGW(0);
    // ---- pass A: validate + count; lane l parses updates l*R .. l*R+R-1
    LWave* LW = (LWave*)&L;
    const uint32_t R = (k + WAVE - 1) / WAVE;
    int err = 0; bool fb = false, nc = false;
    uint32_t sl = 0, dl = 0;
    for (uint32_t r = 0; r < R; r++) {
      const uint32_t i = l * R + r;
      if (i < k) {
        const UpdCount c = w_parse_update(LW, (int)i, false, 0, 0, flags);
        L.uns[i] = (uint16_t)(c.ns > 0xFFFF ? 0xFFFF : c.ns); L.und[i] = (uint16_t)(c.nd > 0xFFFF ? 0xFFFF : c.nd);
        sl += c.ns; dl += c.nd;
        if (c.err && !err) err = c.err;
        fb |= c.fb != 0; nc |= c.nc != 0;
      }
    }
    DIAGW(1);
    const unsigned long long eb = __ballot(err != 0);
    if (eb) st = __shfl(err, __ffsll((long long)eb) - 1, WAVE);
    else if (__ballot(fb)) st = ST_DEFER;
    else {
      (void)wave_exscan(sl, S); (void)wave_exscan(dl, D);
      if (S > (uint32_t)W_S || D > (uint32_t)W_D || ((flags & F_COMPAT_135) && D > 0)) st = ST_DEFER;
      else if (__ballot(nc)) st = ST_NONCANON;
    }
    if (st == ST_OK) {
      // ---- pass B: records
      uint32_t sb, db, tS, tD;
      sb = wave_exscan(sl, tS); db = wave_exscan(dl, tD);
      for (uint32_t r = 0; r < R; r++) {
        const uint32_t i = l * R + r;
        if (i < k) {
          const uint32_t ns = L.uns[i], nd = L.und[i];
          if (ns | nd) w_parse_update(LW, (int)i, true, sb, db, flags);
          sb += ns; db += nd;
        }
      }
      wave_sync();
      DIAGW(2);
      // ---- rank sort (ties by record id; equal struct keys are caught below as overlap)
      for (int pass = 0; pass < 2; pass++) {
        const uint32_t n = pass ? D : S;
        uint64_t mk[W_E]; uint32_t ml[W_E], rk[W_E];
#pragma unroll
        for (int q = 0; q < W_E; q++) {
          const uint32_t j = l + WAVE * q;
          mk[q] = j < n ? (pass ? L.dkey[j] : L.key[j]) : ~0ull; ml[q] = (pass && j < n) ? L.dlen[j] : 0; rk[q] = 0;
        }
        for (uint32_t i = 0; i < n; i++) {
          const uint64_t ki = pass ? L.dkey[i] : L.key[i];
#pragma unroll
          for (int q = 0; q < W_E; q++) rk[q] += (ki < mk[q]) || (ki == mk[q] && i < l + WAVE * q);
        }
        wave_sync();
#pragma unroll
        for (int q = 0; q < W_E; q++) {
          const uint32_t j = l + WAVE * q;
          if (j < n) { if (pass) { L.dkey[rk[q]] = mk[q]; L.dlen[rk[q]] = ml[q]; } else { L.key[rk[q]] = mk[q]; L.sidx[rk[q]] = (uint16_t)j; } }
        }
      }
      for (uint32_t j = l; j < S; j += WAVE) L.runend[j] = 0;
      for (uint32_t j = l; j < D; j += WAVE) L.drunend[j] = 0;
      for (uint32_t j = l; j < W_BLK; j += WAVE) { L.blkcnt[j] = 0; L.segcnt[j] = 0; }
      wave_sync();
      DIAGW(3);
      // ---- classify sorted structs (blocked: lane l owns elements l*W_E .. l*W_E+W_E-1)
      const uint32_t e0 = l * W_E, e1 = min(e0 + W_E, S);
      bool ovl = false;
      uint32_t vmax = 0, nnew = 0;
      for (uint32_t j = e0; j < e1; j++) {
        const uint64_t kj = L.key[j]; const uint32_t r = L.sidx[j];
        uint32_t f = (L.r_flag[r] & 3) == K_GC ? EF_GC : 0;
        if (j == 0) f |= EF_NEWC;
        else {
          const uint64_t kp = L.key[j - 1]; const uint32_t rp = L.sidx[j - 1];
          const uint32_t pend = (uint32_t)kp + L.r_len[rp];
          if ((uint32_t)(kp >> 32) != (uint32_t)(kj >> 32)) f |= EF_NEWC;
          else if ((uint32_t)kj < pend) ovl = true;
          else if ((uint32_t)kj > pend) f |= EF_GAP;
          else {
            const uint32_t ss = L.r_ss[r], sp = L.r_ss[rp];
            if ((ss >> 8) == (sp >> 8) && (ss & 0xFF) == (sp & 0xFF) + 1) f |= EF_SDN;
            if ((f & EF_GC) && (L.r_flag[rp] & 3) == K_GC) f |= EF_CGG;
          }
        }
        if (!(f & EF_CGG)) f |= EF_NONID | EF_T;
        else if (!(f & EF_SDN)) f |= EF_NONID;
        L.eflag[j] = (uint8_t)f;
        if (f & EF_NONID) vmax = j + 1;
        nnew += (f & EF_NEWC) ? 1 : 0;
      }
      uint32_t nsg = 0;
      for (uint32_t j = l; j < D; j += WAVE) nsg += (j == 0 || (L.dkey[j - 1] >> 32) != (L.dkey[j] >> 32)) ? 1u : 0u;
      if (__ballot(ovl)) st = ST_FALLBACK;  // overlapping structs: exact sequential replay
      else if (wave_sum(nnew) > (uint32_t)W_BLK || wave_sum(nsg) > (uint32_t)W_BLK) st = ST_DEFER;
      else {
        wave_sync();
        // last non-identity element <= j (max-scan) and block index (count of NEWC <= j, minus 1)
        uint32_t mex = wave_incl_scan_max(vmax); mex = __shfl_up(mex, 1, WAVE); if (l == 0) mex = 0;
        uint32_t cex = wave_exscan(nnew, nblocks);
        uint32_t hmax = 0, lastnid = mex, blk = cex;
        for (uint32_t j = e0; j < e1; j++) {
          uint32_t f = L.eflag[j];
          if (f & EF_NONID) lastnid = j + 1;
          if (L.eflag[lastnid - 1] & EF_T) f |= EF_EMIT;   // otherwise merged into the previous GC
          L.eflag[j] = (uint8_t)f;
          blk += (f & EF_NEWC) ? 1 : 0;
          L.eblk[j] = (uint8_t)(blk - 1);
          if (f & EF_EMIT) hmax = j + 1;
        }
        uint32_t hex = wave_incl_scan_max(hmax); hex = __shfl_up(hex, 1, WAVE); if (l == 0) hex = 0;
        // per-block struct counts, GC run ends (LDS atomics)
        uint32_t head = hex;
        for (uint32_t j = e0; j < e1; j++) {
          const uint32_t f = L.eflag[j];
          if (f & EF_EMIT) head = j + 1;
          const uint32_t cnt = ((f & EF_GAP) ? 1u : 0u) + ((f & EF_EMIT) ? 1u : 0u);
          if (cnt) atomicAdd(&L.blkcnt[L.eblk[j]], cnt);
          atomicMax(&L.runend[head - 1], (uint32_t)L.key[j] + L.r_len[L.sidx[j]]);
        }
        wave_sync();
        // element sizes -> positions (epos, relative to the struct section)
        uint32_t acc = 0;
        for (uint32_t j = e0; j < e1; j++) {
          const uint32_t f = L.eflag[j];
          const uint64_t kj = L.key[j]; const uint32_t r = L.sidx[j];
          const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(kj >> 32), ck = (uint32_t)kj;
          uint32_t sz = 0;
          if (f & EF_NEWC) sz += vu_len(L.blkcnt[L.eblk[j]]) + vu_len(cl) + vu_len(ck);
          if (f & EF_GAP) { const uint64_t kp = L.key[j - 1]; sz += 1 + vu_len(ck - ((uint32_t)kp + L.r_len[L.sidx[j - 1]])); }
          if (f & EF_EMIT) sz += (f & EF_GC) ? 1 + vu_len(L.runend[j] - ck) : L.r_out[r];
          L.epos[j] = (uint16_t)acc; acc += sz;
        }
        const uint32_t lb0 = wave_exscan(acc, sbytes);
        for (uint32_t j = e0; j < e1; j++) L.epos[j] = (uint16_t)(L.epos[j] + lb0);
        hdr0 = vu_len(nblocks);
        DIAGW(4);
        // ---- delete set: segments (clients, descending) and runs (rule R-DS); lane owns d0 .. d1-1
        const uint32_t d0 = l * W_DE, d1 = min(d0 + W_DE, D);
        uint32_t sn = 0; uint64_t mm = 0;
        for (uint32_t j = d0; j < d1; j++) {
          const bool sg = j == 0 || (L.dkey[j - 1] >> 32) != (L.dkey[j] >> 32);
          L.dflag[j] = sg ? 1 : 0;
          sn += sg ? 1 : 0;
        }
        const uint32_t sex = wave_exscan(sn, nseg);
        uint32_t sidr = sex;
        for (uint32_t j = d0; j < d1; j++) {
          sidr += L.dflag[j] & 1;
          L.dsid[j] = (uint8_t)(sidr - 1);
          const uint64_t v = ((uint64_t)(sidr - 1) << 32) | ((uint32_t)L.dkey[j] + L.dlen[j]);
          mm = v > mm ? v : mm;
        }
        uint64_t dmex = wave_incl_scan_max(mm); dmex = __shfl_up(dmex, 1, WAVE); if (l == 0) dmex = 0;
        uint64_t runmax = dmex; uint32_t rh = 0;
        for (uint32_t j = d0; j < d1; j++) {
          const uint32_t sidj = L.dsid[j];
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
          const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(L.dkey[j] >> 32), ck = (uint32_t)L.dkey[j];
          uint32_t sz = 0;
          if (L.dflag[j] & 1) sz += vu_len(cl) + vu_len(L.segcnt[L.dsid[j]]);
          if (L.dflag[j] & 2) sz += vu_len(ck) + vu_len(L.drunend[j] - ck);
          L.dposs[j] = (uint16_t)dacc; dacc += sz;
        }
        const uint32_t dl0 = wave_exscan(dacc, dsbytes);
        for (uint32_t j = d0; j < d1; j++) L.dposs[j] = (uint16_t)(L.dposs[j] + dl0);
        size = (uint64_t)hdr0 + sbytes + vu_len(nseg) + dsbytes;
      }
    }
  }
  DIAGW(5);
  // ---- look-back (whole wave) -> this document's offset in the packed output
  const uint64_t mysz = st == ST_OK ? size : 0;
  const uint64_t base = lookback(lb, d, mysz, &meta->fault);
  DIAGW(6);
  if (d == n_docs - 1 && l == 0) meta->fast_total = base + mysz;
  if (st == ST_OK && meta->fault) st = ST_DEVICE;
  if (st == ST_OK && base + size > out_cap) st = ST_NOMEM;
  if (l == 0) {
    out_off[d] = base; out_len[d] = st == ST_OK ? size : 0;
    status[d] = st == ST_DEFER ? ST_FALLBACK : st;
    if (st == ST_DEFER) defer_list[atomicAdd(&meta->defer_count, 1u)] = d;
    if (st == ST_FALLBACK) {
      fb_list[atomicAdd(&meta->fb_count, 1u)] = d;
      atomicAdd(&meta->fb_upds, (unsigned long long)k);
      atomicAdd(&meta->fb_bytes, (unsigned long long)nbytes);
    }
  }
  if (st != ST_OK) return;
  uint8_t* o = out + base;
  if (mode == 1) { if (l == 0) { o[0] = 0; o[1] = 0; } return; }
  if (mode == 2) { for (uint64_t i = l; i < nbytes; i += WAVE) o[i] = arena[b0 + i]; return; }
  // ---- emit: lane-contiguous segments
  if (l == 0) { Out w{o, 0}; w.vu(nblocks); }
  const uint32_t e0 = l * W_E, e1 = min(e0 + W_E, S);
  GWriter gw; gw.init(o, hdr0 + (e0 < S ? L.epos[e0] : sbytes));
  for (uint32_t j = e0; j < e1; j++) {
    const uint32_t f = L.eflag[j];
    const uint64_t kj = L.key[j]; const uint32_t r = L.sidx[j];
    const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(kj >> 32), ck = (uint32_t)kj;
    if (f & EF_NEWC) { gw.vu(L.blkcnt[L.eblk[j]]); gw.vu(cl); gw.vu(ck); }
    if (f & EF_GAP) { const uint64_t kp = L.key[j - 1]; gw.b(10); gw.vu(ck - ((uint32_t)kp + L.r_len[L.sidx[j - 1]])); }
    if (f & EF_EMIT) {
      if (f & EF_GC) { gw.b(0); gw.vu(L.runend[j] - ck); }
      else if (!(L.r_flag[r] & 4)) {  // canonical item: input bytes, info bit 0x20 dropped when an origin is set
        const uint32_t s0 = L.r_start[r], n = L.r_blen[r];
        const uint8_t info = L.in[s0];
        gw.b((info & 0xC0) ? (uint8_t)(info & ~0x20) : info);
        for (uint32_t i = 1; i < n; i++) gw.b(L.in[s0 + i]);
      } else {
        gw.flush();
        Cur c{L.in, L.r_start[r], (uint32_t)L.r_start[r] + L.r_blen[r], 0, 0};
        SInfo si; read_struct(c, si, flags);
        Out w{o + gw.pos, 0};
        write_struct(w, L.in, si, cl, ck, 0, false, flags);
        gw.jump(w.n);
      }
    }
  }
  gw.flush();
  const uint32_t dsb = hdr0 + sbytes;
  if (l == 0) { Out w{o + dsb, 0}; w.vu(nseg); }
  const uint32_t d0 = l * W_DE, d1 = min(d0 + W_DE, D);
  GWriter dw; dw.init(o, dsb + vu_len(nseg) + (d0 < D ? L.dposs[d0] : dsbytes));
  for (uint32_t j = d0; j < d1; j++) {
    const uint32_t cl = 0xFFFFFFFFu - (uint32_t)(L.dkey[j] >> 32), ck = (uint32_t)L.dkey[j];
    if (L.dflag[j] & 1) { dw.vu(cl); dw.vu(L.segcnt[L.dsid[j]]); }
    if (L.dflag[j] & 2) { dw.vu(ck); dw.vu(L.drunend[j] - ck); }
  }
  dw.flush();
  DIAGW(7);
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
                                                  int32_t* __restrict__ status, DocMeta* meta, SeqScratch scr, uint64_t out_cap) {
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
    at = meta->fast_total + meta->m_total + atomicAdd(&meta->seq_cursor, (unsigned long long)size);
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
  out_off[d] = at; out_len[d] = st == ST_OK ? size : 0; status[d] = st;
}

}  // namespace ygm

// ======================================================================= launch glue
extern "C" {

using namespace ygm;

#ifdef YGM_DIAG
int ygm_diag_read(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ygm_diag), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) { unsigned long long z[16] = {0}; (void)hipMemcpyToSymbol(HIP_SYMBOL(ygm_diag), z, sizeof z); }
  return 0;
}
#endif

size_t ygm_k_meta_bytes() { return sizeof(DocMeta); }
size_t ygm_k_seq_reader_bytes() { return sizeof(Stream); }
size_t ygm_k_drec_bytes() { return sizeof(DRec); }

int ygm_k_launch_doc(int mode, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                     uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status,
                     unsigned long long* lb, void* meta, uint64_t out_cap, hipStream_t s) {
  const uint32_t tiles = (n_docs + DOC_NT - 1) / DOC_NT;
  if (tiles == 0) return 0;
  if (mode == 0)
    hipLaunchKernelGGL(k_doc<0>, dim3(tiles), dim3(DOC_NT), 0, s, arena, doc_off, sv_arena, sv_off, n_docs, flags, out, out_off, out_len, status, lb, (DocMeta*)meta, out_cap);
  else
    hipLaunchKernelGGL(k_doc<1>, dim3(tiles), dim3(DOC_NT), 0, s, arena, doc_off, sv_arena, sv_off, n_docs, flags, out, out_off, out_len, status, lb, (DocMeta*)meta, out_cap);
  return (int)hipGetLastError();
}

int ygm_k_launch_merge_wave(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, uint32_t flags,
                            uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, unsigned long long* lb, void* meta,
                            uint32_t* defer_list, uint32_t* fb_list, uint64_t out_cap, hipStream_t s) {
  if (n_docs == 0) return 0;
  hipLaunchKernelGGL(k_merge_wave, dim3((n_docs + W_WAVES - 1) / W_WAVES), dim3(WAVE * W_WAVES), 0, s, arena, upd_off, doc_upd, n_docs,
                     flags, out, out_off, out_len, status, lb, (DocMeta*)meta, defer_list, fb_list, out_cap);
  return (int)hipGetLastError();
}

int ygm_k_launch_merge_fast(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs, uint32_t n_docs,
                            uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, unsigned long long* lb,
                            void* meta, uint32_t* fb_list, uint64_t out_cap, hipStream_t s) {
  if (n_docs == 0) return 0;
  hipLaunchKernelGGL(k_merge_fast, dim3(n_docs), dim3(M_NT), 0, s, arena, upd_off, doc_upd, docs, n_docs, flags, out, out_off, out_len,
                     status, lb, (DocMeta*)meta, fb_list, out_cap);
  return (int)hipGetLastError();
}

int ygm_k_launch_merge_seq(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list, uint32_t n_fb,
                           uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta,
                           void* readers, int* order, int* tmp, const uint8_t** ubase, uint32_t* ulen, uint64_t upd_cap,
                           uint32_t* cnt, void* drec, uint64_t byte_cap, uint64_t out_cap, hipStream_t s) {
  if (n_fb == 0) return 0;
  SeqScratch scr{(Stream*)readers, order, tmp, ubase, ulen, cnt, (DRec*)drec, upd_cap, byte_cap};
  hipLaunchKernelGGL(k_merge_seq, dim3((n_fb + 63) / 64), dim3(64), 0, s, arena, upd_off, doc_upd, fb_list, n_fb, flags, out, out_off,
                     out_len, status, (DocMeta*)meta, scr, out_cap);
  return (int)hipGetLastError();
}

}  // extern "C"
