// ygm_snapshot.hip -- doc-normalized snapshot kernels:
//   k_snap_text  : flat-text documents (ygm_snap_text.hpp), one per wave, input + workspace in LDS, into slots;
//                  the documents it leaves take the general path below
//   k_snap_count : per document, the struct / delete-range / client-block counts -> workspace bytes
//   k_snap_scan* : exclusive scan of the workspace sizes (three launches, 256 documents per block)
//   k_snap       : per document, integrate + gc + merge + encode into its workspace's output region
//   k_pend_*     : documents left pending (ST_PEND): their [state, pendingDs, pending structs] packed as three-update
//                  documents for the merge kernels (plan, copy), then the merged bytes' places written back (fix)
// A thread per document keeps the reference's sequential algorithm (YATA integration order matters)
// while 64 documents share a wave; the workspace is per document, so nothing is shared.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ygm_common.hpp"
#include "ygm_snapshot.hpp"
#include "ygm_snap_text.hpp"

namespace ygm {

constexpr int SN_NT = 64;   // one wave per block: documents are independent
constexpr uint32_t SN_DPW = 16;       // documents per wave of the count pass (lanes 0..15)
constexpr uint32_t SN_STAGE = 40960;  // LDS bytes that hold a wave's documents

// The wave's documents [d0, d1) are consecutive in the arena: when their bytes fit, the wave copies them into LDS
// with 16-byte loads and each lane parses its document from there (the codec walks bytes one dependent read at a
// time: ~100 cycles from LDS instead of a global-memory round trip).  Returns the lane's input pointer.
YDEV const uint8_t* snap_stage(uint8_t* stg, const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off, uint32_t d0,
                               uint32_t d1, uint32_t d) {
  const uint64_t a = doc_off[d0], b = doc_off[d1];
  const uint64_t a16 = a & ~15ull;
  const bool staged = b >= a && b - a16 <= SN_STAGE;
  if (staged) {
    const uint4* src = (const uint4*)(arena + a16);
    for (uint32_t c = threadIdx.x; 16u * c < b - a16; c += SN_NT) ((uint4*)stg)[c] = src[c];   // (arena tail padding >= 16)
  }
  __syncthreads();
  if (d >= d1) return nullptr;
  const uint64_t x = doc_off[d];
  return staged && x >= a && doc_off[d + 1] <= b ? stg + (x - a16) : arena + x;
}

// k_snap_text: one document per workgroup (one wave): lane 0 runs the flat-text snapshot (ygm_snap_text.hpp) with
// its workspace in the workgroup's LB bytes of LDS and its input read through the scalar cache (aligned dwords from
// the constant address space: the kernel never writes the arena) -- the integration's dependent chain as LDS round
// trips instead of global ones, the document index wave-uniform so the control flow stays on scalar branches.
// Documents outside the envelope or the workspace are left unclaimed (a second launch with a larger LB, then the
// count / scan / k_snap path).  Outputs go to per-document slots at align16(2 * doc_off[d] + 64 * d), 2n + 48 bytes.
template <uint32_t LB>
__global__ __launch_bounds__(SN_NT) void k_snap_text(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off, uint32_t n_docs,
                                                    uint32_t flags, uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                                                    uint64_t* __restrict__ out_len, int32_t* __restrict__ status, uint8_t* __restrict__ claim,
                                                    unsigned long long* __restrict__ pay, uint32_t again, uint64_t slot_total) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LB];
  const uint32_t d = blockIdx.x;
  if (threadIdx.x != 0 || (again && claim[d])) return;   // (again: the first launch took it)
  const uint64_t a = doc_off[d], b = doc_off[d + 1];
  bool ok = false;
  // (a slot past the caller's region, slot_total = 2 * arena_bytes + 64 * n_docs: left to the general path)
  if (b > a && b - a < 0xFFFFu && snap::al16(2 * a + 64ull * d) + 2 * (b - a) + 48 <= slot_total) {
    const uint32_t n = (uint32_t)(b - a);
    const uint64_t slot = snap::al16(2 * a + 64ull * d);
    snap::OutCap o{out + slot, 0, 2u * n + 48u};
    ok = snapt::snapshot_text(arena + a, n, flags, lds, LB, o) && o.n <= o.cap;
    if (ok) {
      out_off[d] = slot; out_len[d] = o.n; status[d] = ST_OK;
      atomicAdd(pay, (unsigned long long)o.n);
      atomicAdd(pay + 1, 1ull);
    }
  }
  claim[d] = ok ? 1 : 0;
}

__global__ __launch_bounds__(SN_NT) void k_snap_count(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off,
                                                     uint32_t n_docs, uint32_t flags, uint4* __restrict__ cnt,
                                                     uint64_t* __restrict__ need, const uint8_t* __restrict__ claim) {
  __shared__ __attribute__((aligned(16))) uint8_t stg[SN_STAGE + 16];
  const uint32_t d0 = blockIdx.x * SN_DPW, d1 = d0 + SN_DPW < n_docs ? d0 + SN_DPW : n_docs;
  const uint32_t d = d0 + threadIdx.x;
  const uint8_t* in = snap_stage(stg, arena, doc_off, d0, d1, threadIdx.x < SN_DPW ? d : d1);
  if (threadIdx.x >= SN_DPW || d >= n_docs) return;
  if (claim && claim[d]) { cnt[d] = make_uint4(0, 0, 0, 0); need[d] = 0; return; }   // k_snap_text wrote it
  const uint64_t a = doc_off[d], b = doc_off[d + 1];
  uint32_t S = 0, D = 0, C = 0;
  const uint32_t n = b > a && b - a < (1ull << 30) ? (uint32_t)(b - a) : 0u;
  if (n) snap::count_doc(in, n, flags, S, D, C);
  cnt[d] = make_uint4(S, D, C, n);
  need[d] = snap::al16(snap::ws_bytes(snap::caps_of(S, D, C, n)));
}

// exclusive scan of n u64 values in place, total at v[n]: block sums, one block scanning them, apply
__global__ __launch_bounds__(256) void k_snap_scan_sum(const uint64_t* __restrict__ v, uint32_t n, uint64_t* __restrict__ bs) {
  __shared__ uint64_t tmp[256 / WAVE + 1];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint64_t tot;
  (void)block_exscan<256>(i < n ? v[i] : (uint64_t)0, tmp, tot);
  if (threadIdx.x == 0) bs[blockIdx.x] = tot;
}
__global__ __launch_bounds__(1024) void k_snap_scan_top(uint64_t* __restrict__ bs, uint32_t nb) {
  __shared__ uint64_t tmp[1024 / WAVE + 1];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint32_t i = b0 + threadIdx.x;
    uint64_t tot;
    const uint64_t pre = block_exscan<1024>(i < nb ? bs[i] : (uint64_t)0, tmp, tot);
    if (i < nb) bs[i] = carry + pre;
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) bs[nb] = carry;
}
__global__ __launch_bounds__(256) void k_snap_scan_apply(uint64_t* __restrict__ v, uint32_t n, const uint64_t* __restrict__ bs) {
  __shared__ uint64_t tmp[256 / WAVE + 1];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint64_t tot;
  const uint64_t pre = block_exscan<256>(i < n ? v[i] : (uint64_t)0, tmp, tot);
  if (i < n) v[i] = bs[blockIdx.x] + pre;
  if (i == n) v[n] = bs[gridDim.x];
}

__global__ __launch_bounds__(SN_NT) void k_snap(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off, uint32_t n_docs,
                                               uint32_t flags, const uint4* __restrict__ cnt, const uint64_t* __restrict__ ws_off,
                                               uint8_t* __restrict__ ws, uint64_t* __restrict__ out_off, uint64_t* __restrict__ out_len,
                                               int32_t* __restrict__ status, unsigned long long* __restrict__ payload, uint32_t dpw,
                                               const uint8_t* __restrict__ claim, uint64_t base, uint32_t* __restrict__ pend_list,
                                               unsigned int* __restrict__ pend_n) {
  // dpw documents per wave (lanes >= dpw idle): the per-document code diverges from lane to lane, so
  // fewer documents per wave trade SIMD lanes for less serialised divergence and more waves in flight
  __shared__ __attribute__((aligned(16))) uint8_t stg[SN_STAGE + 16];
  const uint32_t d0 = blockIdx.x * dpw, d1 = d0 + dpw < n_docs ? d0 + dpw : n_docs;
  const uint32_t d = d0 + threadIdx.x;
  const uint8_t* in = snap_stage(stg, arena, doc_off, d0, d1, threadIdx.x < dpw ? d : d1);
  uint64_t mine = 0;
  if (threadIdx.x < dpw && d < n_docs && !(claim && claim[d])) {
    const uint4 c = cnt[d];
    const uint64_t a = doc_off[d], b = doc_off[d + 1];
    int st = ST_OK;
    uint32_t oo = 0, ol = 0;
    if (b < a || b - a >= (1ull << 30)) st = ST_INVAL;
    else if (c.w == 0) st = ST_MALFORMED;   // (an empty update: yjs throws reading it)
    else {
      const snap::Caps k = snap::caps_of(c.x, c.y, c.z, c.w);
      st = snap::snapshot_doc(in, c.w, flags, ws + base + ws_off[d], k, oo, ol);
    }
    out_off[d] = base + ws_off[d] + oo;
    out_len[d] = (st == ST_OK || st == snap::ST_PEND) ? ol : 0u;
    status[d] = st;
    if (st == snap::ST_PEND) pend_list[atomicAdd(pend_n, 1u)] = d;   // (rare: one atomic per such document)
    mine = st == ST_OK ? ol : 0u;
  }
  mine = wave_sum(mine);
  if ((threadIdx.x & (WAVE - 1)) == 0 && mine) atomicAdd(payload, (unsigned long long)mine);
}

// ---- pending documents: [state, pendingDs, pending structs] (PendHdr) -> three-update documents for the merge kernels
// plan (one workgroup): document j of the list gets updates 3j .. 3j + 2 at the exclusive prefix of the three lengths
__global__ __launch_bounds__(1024) void k_pend_plan(const uint32_t* __restrict__ list, uint32_t P, const uint8_t* __restrict__ ws,
                                                    const uint64_t* __restrict__ out_off, uint64_t* __restrict__ upd_off,
                                                    uint32_t* __restrict__ doc_upd) {
  __shared__ uint64_t tmp[1024 / WAVE + 1];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t j0 = 0; j0 < P; j0 += 1024) {
    const uint32_t j = j0 + threadIdx.x;
    uint32_t l0 = 0, l1 = 0, l2 = 0;
    if (j < P) {
      const uint8_t* h = ws + out_off[list[j]];   // PendHdr, read by bytes (the region's base need not be aligned)
      auto u32at = [&](uint32_t o) { return (uint32_t)h[o] | ((uint32_t)h[o + 1] << 8) | ((uint32_t)h[o + 2] << 16) | ((uint32_t)h[o + 3] << 24); };
      l0 = u32at(0); l1 = u32at(4); l2 = u32at(8);
    }
    uint64_t tot;
    const uint64_t pre = carry + block_exscan<1024>(j < P ? (uint64_t)l0 + l1 + l2 : (uint64_t)0, tmp, tot);
    if (j < P) { upd_off[3ull * j] = pre; upd_off[3ull * j + 1] = pre + l0; upd_off[3ull * j + 2] = pre + l0 + l1; doc_upd[j] = 3u * j; }
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) { upd_off[3ull * P] = carry; doc_upd[P] = 3u * P; }
}
// copy (a workgroup per document): its three updates to their places in the packed arena
__global__ __launch_bounds__(256) void k_pend_copy(const uint32_t* __restrict__ list, const uint8_t* __restrict__ ws,
                                                   const uint64_t* __restrict__ out_off, const uint64_t* __restrict__ upd_off,
                                                   uint8_t* __restrict__ dst) {
  const uint32_t j = blockIdx.x;
  const uint8_t* src = ws + out_off[list[j]] + sizeof(snap::PendHdr);
  const uint64_t a = upd_off[3ull * j], n = upd_off[3ull * j + 3] - a;
  for (uint64_t i = threadIdx.x; i < n; i += 256) dst[a + i] = src[i];
}
// fix: the merged bytes were appended at `tail` of the output region: each document's place, length and status (pst:
// a status decided before the merge, which wins when non-zero)
__global__ __launch_bounds__(256) void k_pend_fix(const uint32_t* __restrict__ list, uint32_t P, const uint64_t* __restrict__ m_off,
                                                  const uint64_t* __restrict__ m_len, const int32_t* __restrict__ m_st,
                                                  const int32_t* __restrict__ pst, uint64_t tail, uint64_t* __restrict__ out_off,
                                                  uint64_t* __restrict__ out_len, int32_t* __restrict__ status) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= P) return;
  const uint32_t d = list[j];
  const int32_t st = pst && pst[j] ? pst[j] : m_st[j];
  out_off[d] = tail + m_off[j]; out_len[d] = st == ST_OK ? m_len[j] : 0u; status[d] = st;
}

// ---- SyncStep2 of pending documents: encodeStateAsUpdate(doc, sv) = mergeUpdates([writeStateAsUpdate(doc, sv),
// pendingDs, diffUpdate(pending structs, sv)]) (Y@23300).  split: each document's three parts and its state vector
// packed into four arenas (offsets k (P + 1) + j: k = state, pendingDs, pending structs, state vector), for the two
// diffs; join: [diff(state), pendingDs, diff(pending structs)] packed as three-update documents for the merge
YDEV uint32_t pend_len(const uint8_t* h, uint32_t k) {
  return (uint32_t)h[4 * k] | ((uint32_t)h[4 * k + 1] << 8) | ((uint32_t)h[4 * k + 2] << 16) | ((uint32_t)h[4 * k + 3] << 24);
}
__global__ __launch_bounds__(1024) void k_pend_split_plan(const uint32_t* __restrict__ list, uint32_t P, const uint8_t* __restrict__ ws,
                                                          const uint64_t* __restrict__ out_off, const uint64_t* __restrict__ sv_off,
                                                          uint64_t* __restrict__ offs) {
  __shared__ uint64_t tmp[1024 / WAVE + 1];
  __shared__ uint64_t carry[4];
  if (threadIdx.x < 4) carry[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t j0 = 0; j0 < P; j0 += 1024) {
    const uint32_t j = j0 + threadIdx.x;
    uint64_t l[4] = {0, 0, 0, 0};
    if (j < P) {
      const uint32_t d = list[j];
      const uint8_t* h = ws + out_off[d];
      l[0] = pend_len(h, 0); l[1] = pend_len(h, 1); l[2] = pend_len(h, 2); l[3] = sv_off[d + 1] - sv_off[d];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint64_t tot;
      const uint64_t pre = block_exscan<1024>(l[k], tmp, tot);
      if (j < P) offs[(uint64_t)k * (P + 1) + j] = carry[k] + pre;
      __syncthreads();
      if (threadIdx.x == 0) carry[k] += tot;
      __syncthreads();
    }
  }
  if (threadIdx.x < 4) offs[(uint64_t)threadIdx.x * (P + 1) + P] = carry[threadIdx.x];
}
__global__ __launch_bounds__(256) void k_pend_split_copy(const uint32_t* __restrict__ list, uint32_t P, const uint8_t* __restrict__ ws,
                                                         const uint64_t* __restrict__ out_off, const uint8_t* __restrict__ sv,
                                                         const uint64_t* __restrict__ sv_off, const uint64_t* __restrict__ offs,
                                                         uint8_t* __restrict__ da, uint8_t* __restrict__ db, uint8_t* __restrict__ dc,
                                                         uint8_t* __restrict__ dsv) {
  const uint32_t j = blockIdx.x, d = list[j];
  const uint8_t* src = ws + out_off[d] + sizeof(snap::PendHdr);
  uint8_t* const dst[3] = {da, db, dc};
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) {
    const uint64_t a = offs[(uint64_t)k * (P + 1) + j], n = offs[(uint64_t)k * (P + 1) + j + 1] - a;
    for (uint64_t i = threadIdx.x; i < n; i += 256) dst[k][a + i] = src[i];
    src += n;
  }
  const uint64_t a = offs[3ull * (P + 1) + j], n = offs[3ull * (P + 1) + j + 1] - a, s0 = sv_off[d];
  for (uint64_t i = threadIdx.x; i < n; i += 256) dsv[a + i] = sv[s0 + i];
}
__global__ __launch_bounds__(1024) void k_pend_join_plan(uint32_t P, const uint64_t* __restrict__ a_len, const int32_t* __restrict__ a_st,
                                                         const uint64_t* __restrict__ offs, const uint64_t* __restrict__ c_len,
                                                         const int32_t* __restrict__ c_st, uint64_t* __restrict__ upd_off,
                                                         uint32_t* __restrict__ doc_upd, int32_t* __restrict__ pst) {
  __shared__ uint64_t tmp[1024 / WAVE + 1];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t j0 = 0; j0 < P; j0 += 1024) {
    const uint32_t j = j0 + threadIdx.x;
    uint64_t l0 = 0, l1 = 0, l2 = 0;
    if (j < P) {
      l0 = a_st[j] == ST_OK ? a_len[j] : 0u;
      l1 = offs[(P + 1) + j + 1] - offs[(P + 1) + j];
      l2 = c_st[j] == ST_OK ? c_len[j] : 0u;
      pst[j] = a_st[j] != ST_OK ? a_st[j] : c_st[j];
    }
    uint64_t tot;
    const uint64_t pre = carry + block_exscan<1024>(l0 + l1 + l2, tmp, tot);
    if (j < P) { upd_off[3ull * j] = pre; upd_off[3ull * j + 1] = pre + l0; upd_off[3ull * j + 2] = pre + l0 + l1; doc_upd[j] = 3u * j; }
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) { upd_off[3ull * P] = carry; doc_upd[P] = 3u * P; }
}
__global__ __launch_bounds__(256) void k_pend_join_copy(uint32_t P, const uint8_t* __restrict__ ad, const uint64_t* __restrict__ a_off,
                                                        const uint8_t* __restrict__ bd, const uint64_t* __restrict__ offs,
                                                        const uint8_t* __restrict__ cd, const uint64_t* __restrict__ c_off,
                                                        const uint64_t* __restrict__ upd_off, uint8_t* __restrict__ dst) {
  const uint32_t j = blockIdx.x;
  const uint8_t* const src[3] = {ad + a_off[j], bd + offs[(P + 1) + j], cd + c_off[j]};
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) {
    const uint64_t a = upd_off[3ull * j + k], n = upd_off[3ull * j + k + 1] - a;
    for (uint64_t i = threadIdx.x; i < n; i += 256) dst[a + i] = src[k][i];
  }
}

// ---------------------------------------------------------------------------------------------------
// Read-only SyncStep2 (MessageReceiver.ts:156-179): Y.snapshotContainsUpdate(Y.snapshot(doc), update),
// restated from yjs 13.6 (snapshotContainsUpdateV2 -- not in the 13.5.16 bundle): every struct of the
// update (Skips included, in order; the first one past the snapshot's state vector answers false) ends
// at or below the state vector, and merging the update's delete set into the snapshot's leaves it equal.
// The snapshot is given as the document's normalized state (ygm_snapshot_v1 output: its delete set is
// createDeleteSetFromStructStore's, sorted and merged), so the second test is: every update range
// [k, k + l) lies in one snapshot range [a, b) with a <= k and k + l <= b (sortAndMergeDeleteSet).
struct CtSv { uint32_t client, end; };
struct CtDs { uint32_t client, clock, end, pad; };
__global__ __launch_bounds__(SN_NT) void k_cont_count(const uint8_t* __restrict__ st_arena, const uint64_t* __restrict__ st_off,
                                                     uint32_t n_docs, uint32_t flags, uint64_t* __restrict__ need) {
  const uint32_t d = blockIdx.x * SN_NT + threadIdx.x;
  if (d >= n_docs) return;
  const uint64_t a = st_off[d], b = st_off[d + 1];
  uint32_t S = 0, D = 0, C = 0;
  const uint32_t n = b > a && b - a < (1ull << 30) ? (uint32_t)(b - a) : 0u;
  if (n) snap::count_doc(st_arena + a, n, flags, S, D, C);
  need[d] = snap::al16((uint64_t)(C + 1) * sizeof(CtSv)) + snap::al16((uint64_t)(D + 1) * sizeof(CtDs));
}
// ws holds ws_bytes (k_cont_count's size for the document): a snapshot with more blocks or ranges than
// counted (count_doc zeroes its counts past 2^26 structs / ranges) is refused, never written past
YDEV_NI int contains_doc(const uint8_t* sp, uint32_t sn, const uint8_t* up, uint32_t un, uint32_t flags, uint8_t* ws, uint64_t ws_bytes,
                         uint32_t& res) {
  res = 0;
  // the snapshot: state vector (clients of the blocks) and delete set
  Cur c{sp, 0, sn, 0, 0};
  const uint64_t nb = c.vu();
  CtSv* sv = (CtSv*)ws;
  uint32_t nsv = 0;
  for (uint64_t b = 0; b < nb && !c.err; b++) {
    const uint64_t ns = c.vu(), cl = c.vu(); uint64_t ck = c.vu();
    for (uint64_t s = 0; s < ns && !c.err; s++) { SInfo si; read_struct_fast(c, si, flags); ck += si.len; }
    if (cl > 0xFFFFFFFFull || ck > 0xFFFFFFFFull) return snap::ST_UNSUP;
    if (snap::al16((uint64_t)(nsv + 2) * sizeof(CtSv)) + 16u > ws_bytes) return snap::ST_UNSUP;
    sv[nsv].client = (uint32_t)cl; sv[nsv].end = (uint32_t)ck; nsv++;
  }
  if (c.err) return c.err;
  CtDs* ds = (CtDs*)(ws + snap::al16((uint64_t)(nsv + 1) * sizeof(CtSv)));
  uint32_t nds = 0;
  const uint64_t ndc = c.vu();
  for (uint64_t q = 0; q < ndc && !c.err; q++) {
    const uint64_t cl = c.vu(), nr = c.vu();
    for (uint64_t r = 0; r < nr && !c.err; r++) {
      const uint64_t ck = c.vu(), ln = c.vu();
      if (cl > 0xFFFFFFFFull || ck + ln > 0xFFFFFFFFull) return snap::ST_UNSUP;
      if ((uint64_t)((uint8_t*)(ds + nds + 1) - ws) > ws_bytes) return snap::ST_UNSUP;
      ds[nds].client = (uint32_t)cl; ds[nds].clock = (uint32_t)ck; ds[nds].end = (uint32_t)(ck + ln); nds++;
    }
  }
  if (c.err) return c.err;
  // the update: structs in order, then its delete set
  Cur u{up, 0, un, 0, 0};
  const uint64_t ub = u.vu();
  for (uint64_t b = 0; b < ub && !u.err; b++) {
    const uint64_t ns = u.vu(), cl = u.vu(); uint64_t ck = u.vu();
    if (u.err) break;
    uint64_t have = 0;
    for (uint32_t i = 0; i < nsv; i++) if (sv[i].client == cl) have = sv[i].end;
    for (uint64_t s = 0; s < ns && !u.err; s++) {
      SInfo si; read_struct_fast(u, si, flags);
      if (u.err) break;
      ck += si.len;
      if (have < ck) return ST_OK;   // res = 0: a struct past the snapshot
    }
  }
  if (u.err) return u.err;
  const uint64_t udc = u.vu();
  for (uint64_t q = 0; q < udc && !u.err; q++) {
    const uint64_t cl = u.vu(), nr = u.vu();
    for (uint64_t r = 0; r < nr && !u.err; r++) {
      const uint64_t k = u.vu(), l = u.vu();
      if (u.err) break;
      bool cov = false;
      for (uint32_t i = 0; i < nds && !cov; i++) cov = ds[i].client == cl && ds[i].clock <= k && k + l <= ds[i].end;
      if (!cov) { res = 0; return ST_OK; }
    }
  }
  if (u.err) return u.err;
  res = 1;
  return ST_OK;
}
__global__ __launch_bounds__(SN_NT) void k_cont(const uint8_t* __restrict__ st_arena, const uint64_t* __restrict__ st_off,
                                               const uint8_t* __restrict__ up_arena, const uint64_t* __restrict__ up_off, uint32_t n_docs,
                                               uint32_t flags, const uint64_t* __restrict__ ws_off, uint8_t* __restrict__ ws,
                                               uint8_t* __restrict__ out, uint64_t* __restrict__ out_off, uint64_t* __restrict__ out_len,
                                               int32_t* __restrict__ status) {
  const uint32_t d = blockIdx.x * SN_NT + threadIdx.x;
  if (d >= n_docs) return;
  const uint64_t a = st_off[d], b = st_off[d + 1], ua = up_off[d], ub = up_off[d + 1];
  uint32_t res = 0;
  int st;
  if (b < a || ub < ua || b - a >= (1ull << 30) || ub - ua >= (1ull << 30)) st = ST_INVAL;
  else st = contains_doc(st_arena + a, (uint32_t)(b - a), up_arena + ua, (uint32_t)(ub - ua), flags, ws + ws_off[d], ws_off[d + 1] - ws_off[d], res);
  out[d] = (uint8_t)res;
  out_off[d] = d; out_len[d] = st == ST_OK ? 1u : 0u; status[d] = st;
}

}  // namespace ygm

using namespace ygm;

extern "C" {

static int snap_rc(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { fprintf(stderr, "ygm: %s: %s\n", fn, hipGetErrorString(e)); return -1; }
  return 0;
}

// phase 1: counts and the scanned workspace offsets (ws_off: n_docs + 1 entries, total at [n_docs];
// bs: ceil(n / 256) + 1 scratch entries)
int ygm_k_launch_snap_text(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                           uint64_t* out_len, int32_t* status, uint8_t* claim, unsigned long long* pay, int again, uint64_t slot_total, hipStream_t s) {
  if (n_docs == 0) return 0;
  // again == 0: 6 KiB of LDS per document (209 parts); again == 1: 24 KiB for the documents the first launch left.
  // YGM_SNAP_TEXT="KiB" picks another measured size for the first launch.
  if (again) {
    hipLaunchKernelGGL((k_snap_text<24576>), dim3(n_docs), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, out, out_off, out_len, status,
                       claim, pay, 1u, slot_total);
    return snap_rc(__func__);
  }
  const char* env = getenv("YGM_SNAP_TEXT");
  const int lb = env ? atoi(env) : 6;
#define SNT(L) if (lb == L) { hipLaunchKernelGGL((k_snap_text<L * 1024>), dim3(n_docs), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, out, \
                                                   out_off, out_len, status, claim, pay, 0u, slot_total); return snap_rc(__func__); }
  SNT(4) SNT(5) SNT(8)
#undef SNT
  if (lb == 53) { hipLaunchKernelGGL((k_snap_text<5376>), dim3(n_docs), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, out, out_off, out_len, status,
                                     claim, pay, 0u, slot_total); return snap_rc(__func__); }
  hipLaunchKernelGGL((k_snap_text<6144>), dim3(n_docs), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, out, out_off, out_len, status, claim,
                     pay, 0u, slot_total);
  return snap_rc(__func__);
}
int ygm_k_launch_snap_plan(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, void* cnt, uint64_t* ws_off,
                           uint64_t* bs, const uint8_t* claim, hipStream_t s) {
  if (n_docs == 0) return 0;
  const uint32_t g = (n_docs + SN_DPW - 1) / SN_DPW, nb = (n_docs + 1 + 255) / 256;
  hipLaunchKernelGGL(k_snap_count, dim3(g), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, (uint4*)cnt, ws_off, claim);
  hipLaunchKernelGGL(k_snap_scan_sum, dim3(nb), dim3(256), 0, s, (const uint64_t*)ws_off, n_docs, bs);
  hipLaunchKernelGGL(k_snap_scan_top, dim3(1), dim3(1024), 0, s, bs, nb);
  hipLaunchKernelGGL(k_snap_scan_apply, dim3(nb), dim3(256), 0, s, ws_off, n_docs, (const uint64_t*)bs);
  return snap_rc(__func__);
}
// exclusive scan of v[0..n) in place, total at v[n] (bs: ceil((n + 1) / 256) + 1 scratch entries)
int ygm_k_launch_scan(uint64_t* v, uint32_t n, uint64_t* bs, hipStream_t s) {
  if (n == 0) return 0;
  const uint32_t nb = (n + 1 + 255) / 256;
  hipLaunchKernelGGL(k_snap_scan_sum, dim3(nb), dim3(256), 0, s, (const uint64_t*)v, n, bs);
  hipLaunchKernelGGL(k_snap_scan_top, dim3(1), dim3(1024), 0, s, bs, nb);
  hipLaunchKernelGGL(k_snap_scan_apply, dim3(nb), dim3(256), 0, s, v, n, (const uint64_t*)bs);
  return snap_rc(__func__);
}
// phase 2: the snapshots (ws sized from ws_off[n_docs])
int ygm_k_launch_snap(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, const void* cnt, const uint64_t* ws_off,
                      uint8_t* ws, uint64_t* out_off, uint64_t* out_len, int32_t* status, unsigned long long* payload, const uint8_t* claim,
                      uint64_t base, uint32_t* pend_list, unsigned int* pend_n, hipStream_t s) {
  if (n_docs == 0) return 0;
  const char* env = getenv("YGM_SNAP_DPW");
  uint32_t dpw = env ? (uint32_t)atoi(env) : 16u;
  if (dpw < 1 || dpw > (uint32_t)SN_NT) dpw = 16u;
  const uint32_t g = (n_docs + dpw - 1) / dpw;
  hipLaunchKernelGGL(k_snap, dim3(g), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, (const uint4*)cnt, ws_off, ws, out_off, out_len,
                     status, payload, dpw, claim, base, pend_list, pend_n);
  return snap_rc(__func__);
}
int ygm_k_launch_pend_plan(const uint32_t* list, uint32_t P, const uint8_t* ws, const uint64_t* out_off, uint64_t* upd_off, uint32_t* doc_upd,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_pend_plan, dim3(1), dim3(1024), 0, s, list, P, ws, out_off, upd_off, doc_upd);
  return snap_rc(__func__);
}
int ygm_k_launch_pend_copy(const uint32_t* list, uint32_t P, const uint8_t* ws, const uint64_t* out_off, const uint64_t* upd_off, uint8_t* dst,
                           hipStream_t s) {
  if (P == 0) return 0;
  hipLaunchKernelGGL(k_pend_copy, dim3(P), dim3(256), 0, s, list, ws, out_off, upd_off, dst);
  return snap_rc(__func__);
}
int ygm_k_launch_pend_fix(const uint32_t* list, uint32_t P, const uint64_t* m_off, const uint64_t* m_len, const int32_t* m_st,
                          const int32_t* pst, uint64_t tail, uint64_t* out_off, uint64_t* out_len, int32_t* status, hipStream_t s) {
  if (P == 0) return 0;
  hipLaunchKernelGGL(k_pend_fix, dim3((P + 255) / 256), dim3(256), 0, s, list, P, m_off, m_len, m_st, pst, tail, out_off, out_len, status);
  return snap_rc(__func__);
}
int ygm_k_launch_pend_split(const uint32_t* list, uint32_t P, const uint8_t* ws, const uint64_t* out_off, const uint8_t* sv,
                            const uint64_t* sv_off, uint64_t* offs, uint8_t* da, uint8_t* db, uint8_t* dc, uint8_t* dsv, int pass,
                            hipStream_t s) {
  if (P == 0) return 0;
  if (pass == 0) hipLaunchKernelGGL(k_pend_split_plan, dim3(1), dim3(1024), 0, s, list, P, ws, out_off, sv_off, offs);
  else hipLaunchKernelGGL(k_pend_split_copy, dim3(P), dim3(256), 0, s, list, P, ws, out_off, sv, sv_off, (const uint64_t*)offs, da, db, dc, dsv);
  return snap_rc(__func__);
}
int ygm_k_launch_pend_join(uint32_t P, const uint8_t* ad, const uint64_t* a_off, const uint64_t* a_len, const int32_t* a_st, const uint8_t* bd,
                           const uint64_t* offs, const uint8_t* cd, const uint64_t* c_off, const uint64_t* c_len, const int32_t* c_st,
                           uint64_t* upd_off, uint32_t* doc_upd, int32_t* pst, uint8_t* dst, int pass, hipStream_t s) {
  if (P == 0) return 0;
  if (pass == 0) hipLaunchKernelGGL(k_pend_join_plan, dim3(1), dim3(1024), 0, s, P, a_len, a_st, offs, c_len, c_st, upd_off, doc_upd, pst);
  else hipLaunchKernelGGL(k_pend_join_copy, dim3(P), dim3(256), 0, s, P, ad, a_off, bd, offs, cd, c_off, (const uint64_t*)upd_off, dst);
  return snap_rc(__func__);
}

// read-only SyncStep2 containment: workspace plan (the snapshot scan), then one thread per document
int ygm_k_launch_cont_plan(const uint8_t* st_arena, const uint64_t* st_off, uint32_t n_docs, uint32_t flags, uint64_t* ws_off, uint64_t* bs,
                           hipStream_t s) {
  if (n_docs == 0) return 0;
  const uint32_t g = (n_docs + SN_NT - 1) / SN_NT, nb = (n_docs + 1 + 255) / 256;
  hipLaunchKernelGGL(k_cont_count, dim3(g), dim3(SN_NT), 0, s, st_arena, st_off, n_docs, flags, ws_off);
  hipLaunchKernelGGL(k_snap_scan_sum, dim3(nb), dim3(256), 0, s, (const uint64_t*)ws_off, n_docs, bs);
  hipLaunchKernelGGL(k_snap_scan_top, dim3(1), dim3(1024), 0, s, bs, nb);
  hipLaunchKernelGGL(k_snap_scan_apply, dim3(nb), dim3(256), 0, s, ws_off, n_docs, (const uint64_t*)bs);
  return snap_rc(__func__);
}
int ygm_k_launch_cont(const uint8_t* st_arena, const uint64_t* st_off, const uint8_t* up_arena, const uint64_t* up_off, uint32_t n_docs,
                      uint32_t flags, const uint64_t* ws_off, uint8_t* ws, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                      int32_t* status, hipStream_t s) {
  if (n_docs == 0) return 0;
  const uint32_t g = (n_docs + SN_NT - 1) / SN_NT;
  hipLaunchKernelGGL(k_cont, dim3(g), dim3(SN_NT), 0, s, st_arena, st_off, up_arena, up_off, n_docs, flags, ws_off, ws, out, out_off, out_len,
                     status);
  return snap_rc(__func__);
}

}  // extern "C"
