// ygm_v2.hip -- update-V2 kernels: one lane per update / document runs the transcoders of
// ygm_v2.hpp in two passes (sizes, then bytes at scanned offsets).
//   k_v21_count / k_v21_write : V2 -> V1 per update (merge: updates of single-input documents are skipped --
//                               mergeUpdatesV2 returns a lone input as it is); the wave's bytes staged in LDS, the
//                               register-resident transcoder (ygm_v21_fast.hpp) first
//   k_v12_count / k_v12_write : V1 -> V2 per document, with the document's final status (the V2 inputs'
//                               transcoding statuses, then the V1 operation's), or the passthrough copy
//   k_v2_status               : SV: a V2 input's transcoding status over the V1 kernel's
// The lanes of a wave take different paths through the byte codec; documents are independent, so nothing
// is shared and the wave only pays divergence.  The V1 operation between the passes is the engine's V1
// cascade, unchanged.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ygm_common.hpp"
#include "ygm_v2.hpp"
#include "ygm_v2_fast.hpp"
#include "ygm_v21_fast.hpp"

namespace ygm {

constexpr int V2_NT = 64;

YDEV bool is_throw(int st) { return st == ST_MALFORMED || st == ST_RANGE || st == ST_SURROGATE || st == ST_DEPTH; }

// the document of update u (doc_upd: n_docs + 1 non-decreasing update offsets)
YDEV uint32_t doc_of(const uint32_t* doc_upd, uint32_t n_docs, uint32_t u) {
  uint32_t lo = 0, hi = n_docs;   // last d with doc_upd[d] <= u
  while (hi - lo > 1) { const uint32_t m = (lo + hi) / 2; if (doc_upd[m] <= u) lo = m; else hi = m; }
  return lo;
}

// V2 -> V1, one lane per update, in two kernels per pass:
//   k_v21f<W>   : the wave's updates are consecutive in the arena, so the wave copies their bytes into LDS with
//                 16-byte loads and each lane runs the register-resident transcoder (ygm_v21_fast.hpp: text-log
//                 shapes, <= 128 bytes); the updates it takes are claimed (cl[u] = 1)
//   k_v21_*     : the general transcoder (v2::v21, decoder state in scratch, ~250 VGPRs) for the unclaimed rest
// The size pass and the write pass make the same choice per update, so sizes and bytes agree.
constexpr uint32_t V21_STG = 8192;
template <bool W>
__global__ __launch_bounds__(V2_NT) void k_v21f(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off, uint32_t n_upd,
                                               const uint32_t* __restrict__ doc_upd, uint32_t n_docs, uint32_t mode,
                                               uint64_t* __restrict__ len_or_off, int32_t* __restrict__ st, uint8_t* __restrict__ cl,
                                               uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t stg[V21_STG + 16];
  const uint32_t u0 = blockIdx.x * V2_NT, u1 = u0 + V2_NT < n_upd ? u0 + V2_NT : n_upd;
  const uint64_t a0 = upd_off[u0], b0 = upd_off[u1], a16 = a0 & ~15ull;
  const bool staged = b0 >= a0 && b0 - a16 <= V21_STG;
  if (staged) {
    const uint4* src = (const uint4*)(arena + a16);
    for (uint32_t c = threadIdx.x; 16u * c < b0 - a16; c += V2_NT) ((uint4*)stg)[c] = src[c];   // (arena tail padding >= 16)
  }
  __syncthreads();
  const uint32_t u = u0 + threadIdx.x;
  if (u >= n_upd) return;
  if (W) {
    if (!cl[u]) return;
    const uint64_t a = upd_off[u], b = upd_off[u + 1];
    if (len_or_off[u + 1] == len_or_off[u]) return;
    const v21f::Src<const uint8_t*> s{stg + (a - a16)};
    v21f::BOut<uint8_t*> o{out + len_or_off[u], 0};
    (void)v21f::v21_fast(s, (uint32_t)(b - a), mode, o);
    return;
  }
  uint8_t c = 0;
  if (doc_upd) {
    const uint32_t d = doc_of(doc_upd, n_docs, u);
    if (doc_upd[d + 1] - doc_upd[d] == 1) { len_or_off[u] = 0; st[u] = ST_OK; cl[u] = 1; return; }
  }
  const uint64_t a = upd_off[u], b = upd_off[u + 1];
  if (staged && b >= a && b - a <= v21f::F21_MAX) {
    const v21f::Src<const uint8_t*> s{stg + (a - a16)};
    v21f::BOut<uint8_t*> o{nullptr, 0};
    if (v21f::v21_fast(s, (uint32_t)(b - a), mode, o)) { len_or_off[u] = o.n; st[u] = ST_OK; c = 1; }
  }
  cl[u] = c;
}

__global__ __launch_bounds__(V2_NT) void k_v21_count(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off, uint32_t n_upd,
                                                    const uint32_t* __restrict__ doc_upd, uint32_t n_docs, uint32_t mode, uint32_t flags,
                                                    uint64_t* __restrict__ len, int32_t* __restrict__ st, const uint8_t* __restrict__ cl) {
  const uint32_t u = blockIdx.x * V2_NT + threadIdx.x;
  if (u >= n_upd || (cl && cl[u])) return;
  if (doc_upd) {
    const uint32_t d = doc_of(doc_upd, n_docs, u);
    if (doc_upd[d + 1] - doc_upd[d] == 1) { len[u] = 0; st[u] = ST_OK; return; }
  }
  const uint64_t a = upd_off[u], b = upd_off[u + 1];
  if (b < a || b - a >= (1ull << 30)) { len[u] = 0; st[u] = ST_INVAL; return; }
  Out o{nullptr, 0};
  const int e = v2::v21(arena + a, (uint32_t)(b - a), a, mode, flags, o);
  len[u] = e ? 0u : o.n;
  st[u] = e;
}
__global__ __launch_bounds__(V2_NT) void k_v21_write(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ upd_off, uint32_t n_upd,
                                                    uint32_t mode, uint32_t flags, const uint64_t* __restrict__ off,
                                                    const int32_t* __restrict__ st, uint8_t* __restrict__ out, const uint8_t* __restrict__ cl) {
  const uint32_t u = blockIdx.x * V2_NT + threadIdx.x;
  if (u >= n_upd || (cl && cl[u]) || st[u] != ST_OK || off[u + 1] == off[u]) return;
  const uint64_t a = upd_off[u], b = upd_off[u + 1];
  Out o{out + off[u], 0};
  (void)v2::v21(arena + a, (uint32_t)(b - a), a, mode, flags, o);
}

// per document: final status and V2 size.  merge (doc_upd != null): a single-input document is passed
// through (L[0] = ~0); otherwise a throw in any input's transcoding wins over a refusal, then the V1
// merge's status.  diff / public V1 -> V2 (doc_upd == null): ust[d] (if given), then v1_st[d] (if given).
__global__ __launch_bounds__(V2_NT) void k_v12_count(const uint8_t* __restrict__ v1, const uint64_t* __restrict__ v1_off,
                                                    const uint64_t* __restrict__ v1_len, const int32_t* __restrict__ v1_st,
                                                    const uint8_t* __restrict__ v2a, uint64_t v2n, const uint64_t* __restrict__ upd_off,
                                                    const uint32_t* __restrict__ doc_upd, const int32_t* __restrict__ ust, uint32_t n_docs,
                                                    uint32_t mode, uint32_t flags, uint32_t* __restrict__ L, uint64_t* __restrict__ tot,
                                                    int32_t* __restrict__ st, const uint8_t* __restrict__ claim) {
  const uint32_t d = blockIdx.x * V2_NT + threadIdx.x;
  if (d >= n_docs) return;
  if (claim && claim[d]) { tot[d] = 0; return; }   // k_v12_fast wrote it (status, offset, length)
  uint32_t* Ld = L + (size_t)d * v2::C_N;
  int s = ST_OK;
  if (doc_upd) {
    const uint32_t u0 = doc_upd[d], u1 = doc_upd[d + 1];
    if (u1 - u0 == 1) { Ld[0] = 0xFFFFFFFFu; tot[d] = upd_off[u1] - upd_off[u0]; st[d] = ST_OK; return; }
    int refuse = ST_OK;
    for (uint32_t u = u0; u < u1 && !s; u++) { const int e = ust[u]; if (is_throw(e) || e == ST_INVAL) s = e; else if (e && !refuse) refuse = e; }
    if (!s) s = refuse;
  } else if (ust) s = ust[d];
  if (!s && v1_st) s = v1_st[d];
  uint64_t t = 0;
  if (!s) {
    const uint64_t len = v1_len ? v1_len[d] : v1_off[d + 1] - v1_off[d];
    if (len >= (1ull << 30)) s = ST_INVAL;
    else {
      v2::Enc2 w; v2::enc_init(w);
      s = v2::v12_body(v1 + v1_off[d], (uint32_t)len, v2a, v2n, mode, flags, w);
      for (int i = 0; i < v2::C_N; i++) Ld[i] = w.o[i].n;
      if (!s) t = v2::v2_total(Ld);
    }
  }
  Ld[0] = s ? 0u : Ld[0];
  tot[d] = s ? 0u : t;
  st[d] = s;
}
__global__ __launch_bounds__(V2_NT) void k_v12_write(const uint8_t* __restrict__ v1, const uint64_t* __restrict__ v1_off,
                                                    const uint64_t* __restrict__ v1_len, const uint8_t* __restrict__ v2a, uint64_t v2n,
                                                    const uint64_t* __restrict__ upd_off, const uint32_t* __restrict__ doc_upd, uint32_t n_docs,
                                                    uint32_t mode, uint32_t flags, const uint32_t* __restrict__ L,
                                                    const uint64_t* __restrict__ off, int32_t* __restrict__ st, uint8_t* __restrict__ out,
                                                    uint64_t* __restrict__ out_len, const uint8_t* __restrict__ claim, uint64_t base,
                                                    uint64_t* __restrict__ fo) {
  const uint32_t d = blockIdx.x * V2_NT + threadIdx.x;
  if (d >= n_docs || (claim && claim[d])) return;
  const uint32_t* Ld = L + (size_t)d * v2::C_N;
  const uint64_t o0 = base + off[d], n = off[d + 1] - off[d];
  fo[d] = o0;
  out_len[d] = st[d] == ST_OK ? n : 0u;
  if (st[d] != ST_OK) return;
  if (doc_upd && Ld[0] == 0xFFFFFFFFu) {   // single input: as it is
    const uint8_t* src = v2a + upd_off[doc_upd[d]];
    for (uint64_t i = 0; i < n; i++) out[o0 + i] = src[i];
    return;
  }
  const uint64_t len = v1_len ? v1_len[d] : v1_off[d + 1] - v1_off[d];
  const int e = v2::v12_write(v1 + v1_off[d], (uint32_t)len, v2a, v2n, mode, flags, Ld, out + o0);
  if (e) { st[d] = ST_DEVICE; out_len[d] = 0; }   // (the count pass took the same path: cannot happen)
}
// V1 -> V2 of the documents in the fast encoder's shape (ygm_v2_fast.hpp): D documents per wave, nine lanes per
// document, one V2 column per lane.  Each document's V1 bytes are staged in LDS by 16-byte loads with its terminator
// masks; the nine lanes of a document walk the same bytes (one decode stream, LDS reads broadcast) and each encodes
// its own column -- a count pass, the layout from the nine lengths, a write pass that stores the column straight
// into the document's slot (merge_slot of its V2 input bytes, as the V1 kernels place outputs: no scan, no
// cross-document dependency).  The small tier stages documents of <= 3.25 KB (five per wave, 45 lanes busy: the sizing
// below), a
// second launch (D = 2, 7 KB) the larger ones.  claim[d] = 1 for a document done here; the general kernels take
// the rest (their outputs after the slot region).
// a lane's column from its scratch (16-byte aligned, CAP a multiple of 16) to its place in the slot: 16-byte loads,
// each a whole piece of the column before its stores (a byte loop reloading the scratch after every store to the
// slot -- which may alias it for the compiler -- waited on each load: ~1.5 ms per 10 000 documents)
YDEV void v12f_copy_col(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, uint32_t n) {
  typedef unsigned int cu32x4 __attribute__((ext_vector_type(4)));
  uint32_t i = 0;
  for (; i + 16u <= n; i += 16u) { const cu32x4 v = *(const cu32x4*)(s + i); __builtin_memcpy(d + i, &v, 16); }
  if (i < n) {   // (i is a multiple of 16 below n <= CAP: the piece stays inside the lane's region)
    const cu32x4 v = *(const cu32x4*)(s + i);
    for (uint32_t k = 0; k < n - i; k++) {
      const uint32_t w = k < 4u ? v.x : k < 8u ? v.y : k < 12u ? v.z : v.w;
      d[i + k] = (uint8_t)(w >> (8u * (k & 3u)));
    }
  }
}
typedef __attribute__((address_space(3))) uint8_t FL8;
typedef __attribute__((address_space(3))) uint64_t FL64;
typedef unsigned int fu32x4 __attribute__((ext_vector_type(4)));
template <int FIN>
struct alignas(16) V2FDoc {
  static constexpr uint32_t INB = FIN + 128;   // the 0..15 byte shift, the update, 64+ bytes of zeros
  uint8_t in[INB];
  uint64_t m[INB / 64 + 2];
};
YDEV uint64_t v2_slot(uint64_t b0, uint32_t d) { return (2 * b0 + 64ull * d + 15) & ~15ull; }
template <int D, int FIN>
__global__ __launch_bounds__(64) void k_v12_fast(const uint8_t* __restrict__ v1, const uint64_t* __restrict__ v1_off,
                                                 const uint64_t* __restrict__ v1_len, const int32_t* __restrict__ v1_st,
                                                 const uint64_t* __restrict__ slot_off, const uint32_t* __restrict__ doc_upd,
                                                 const int32_t* __restrict__ ust, uint32_t n_docs, uint8_t* __restrict__ out,
                                                 uint64_t* __restrict__ fo, uint64_t* __restrict__ olen, int32_t* __restrict__ ost,
                                                 uint8_t* __restrict__ claim, unsigned long long* __restrict__ payload, int second,
                                                 uint8_t* __restrict__ scr, uint64_t slot_total) {
  static_assert(D * v2f::FC_N <= WAVE, "nine lanes per document");
  typedef V2FDoc<FIN> Doc;
  constexpr uint32_t CAP = FIN + 64;   // scratch bytes per column (a column past it: the document goes on)
  __shared__ Doc S[D];
  const uint32_t l = threadIdx.x, g = l / v2f::FC_N, col = l % v2f::FC_N;   // lane l: document g, column col
  // this lane's column scratch (persistent grid: a wave reuses its own region)
  uint8_t* cs = scr + ((size_t)blockIdx.x * D * v2f::FC_N + (g < (uint32_t)D ? g * v2f::FC_N + col : 0u)) * CAP;
  for (uint32_t grp = blockIdx.x; (uint64_t)grp * D < n_docs; grp += gridDim.x) {
    uint32_t g_sh = 0, g_n = 0;              // lanes of document g: its staged shift and end
    bool g_ok = false;
    uint64_t g_slot = 0, g_cap = 0;
    __syncthreads();                          // (the previous group's staged bytes are no longer read)
    for (int j = 0; j < D; j++) {
      const uint32_t d = grp * D + (uint32_t)j;
      if (d >= n_docs) break;
      // eligibility: every input transcoded, the V1 operation OK, not a passthrough, staged size (second launch:
      // only what the first one left)
      bool bad = second && claim[d];
      uint64_t b0 = 0, nb = 0;
      if (!bad) {
        if (doc_upd) {
          const uint32_t u0 = doc_upd[d], u1 = doc_upd[d + 1];
          bad = u1 - u0 < 2u;
          for (uint32_t u = u0 + l; u < u1 && !bad; u += WAVE) bad = ust[u] != ST_OK;
          b0 = slot_off[u0]; nb = slot_off[u1] - b0;
        } else {
          bad = ust && ust[d] != ST_OK;
          b0 = slot_off[d]; nb = slot_off[d + 1] - b0;
        }
      }
      if (v1_st && v1_st[d] != ST_OK) bad = true;
      const uint64_t a = v1_off[d], len = v1_len ? v1_len[d] : v1_off[d + 1] - a;
      if (len > (uint64_t)FIN || len == 0) bad = true;
      if (v2_slot(b0, d) + 2 * nb + 48 > slot_total) bad = true;   // a slot past the caller's region: the general pass
      if (__ballot(bad)) { if (l == 0 && !(second && claim[d])) claim[d] = 0; continue; }
      // stage: 16-byte loads from the aligned base (the V1 arenas carry >= 16 bytes of readable tail)
      const uint32_t sh = (uint32_t)(a & 15u), n = sh + (uint32_t)len;
      const fu32x4* src = (const fu32x4*)(v1 + (a & ~15ull));
      const uint32_t nw = (n + 63u) / 64u + 1u;   // mask words read: up to the one past the update's last byte
      for (uint32_t c = l; c < 4u * nw; c += WAVE) {
        fu32x4 v = {0u, 0u, 0u, 0u};
        if (c * 16u < n) v = src[c];
        *(fu32x4*)(S[j].in + 16u * c) = v;
      }
      if (g == (uint32_t)j) { g_ok = true; g_sh = sh; g_n = n; g_slot = v2_slot(b0, d); g_cap = 2 * nb + 48; }
    }
    __syncthreads();
    for (int j = 0; j < D; j++) {
      const uint32_t nj = (uint32_t)__shfl((int)g_n, j * (int)v2f::FC_N);
      const uint32_t nw = nj ? (nj + 63u) / 64u + 1u : 0u;
      for (uint32_t k = l; k <= nw && nw; k += WAVE) S[j].m[k] = v2f::f_mask_word((FL8*)S[j].in, k);
    }
    __syncthreads();
    if (g < (uint32_t)D && g_ok) {
      const uint32_t d = grp * D + g;
      const v2f::FSrc<FL8*, FL64*> src{(FL8*)S[g].in, (FL64*)S[g].m};
      v2f::FCS c;
      // ONE pass: the column into this lane's scratch, then the layout from the nine lengths, then the copy
      bool ok = v2f::f_col_run(src, g_sh, g_n, col, cs, 0u, CAP, c);
      uint32_t L[v2f::FC_N], base[v2f::FC_N];
#pragma unroll
      for (int q = 0; q < (int)v2f::FC_N; q++) L[q] = (uint32_t)__shfl((int)c.n, (int)(g * v2f::FC_N) + q, WAVE);
      bool fits = true;
#pragma unroll
      for (int q = 0; q < (int)v2f::FC_N; q++) fits = fits && L[q] <= CAP;
      const uint32_t total = v2f::fc_layout((uint8_t*)nullptr, L, base);
      ok = ok && fits && ((total + 15u) & ~15u) <= g_cap;
      if (ok) {
        uint8_t* o = out + g_slot;
        if (col == 0u) (void)v2f::fc_layout(o, L, base);
        uint32_t mb = base[0];
#pragma unroll
        for (int q = 1; q < (int)v2f::FC_N; q++) mb = col == (uint32_t)q ? base[q] : mb;
        v12f_copy_col(o + mb, cs, c.n);
      }
      if (col == 0u) {
        if (ok) {
          fo[d] = g_slot; olen[d] = total; ost[d] = ST_OK; claim[d] = 1;
          atomicAdd(payload, (unsigned long long)total);   // payload[0]: bytes, payload[1]: documents claimed
          atomicAdd(payload + 1, 1ull);
        } else if (!second) claim[d] = 0;
      }
    }
  }
}

// persistent grids: the waves resident at once (their column scratch is reused group after group)
template <int D, int FIN>
static uint32_t v12f_grid() {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_v12_fast<D, FIN>, WAVE, 0) != hipSuccess || cus <= 0 || per <= 0)
    return 2048u;
  return (uint32_t)(cus * per);
}
template <int D, int FIN>
static size_t v12f_scratch() { return (size_t)v12f_grid<D, FIN>() * D * v2f::FC_N * (FIN + 64); }
// small tier: five documents of <= 3.25 KB per wave (19.5 KB of LDS: eight waves per CU, 10 240 documents resident --
// a batch of 10 000 merged C2 logs, <= 3 023 bytes each, in one round; four of <= 3.5 KB: 9 216 resident, two rounds,
// 1.83 against 1.22 ms for the v2 block; six / seven of <= 3 KB per wave, also one round: 1.27 / 1.28 ms; one per
// wave: 30 % slower)
constexpr int V12F_D = 5, V12F_FS = 3328;

__global__ __launch_bounds__(256) void k_v2_status(const int32_t* __restrict__ ust, uint32_t n, int32_t* __restrict__ status,
                                                  uint64_t* __restrict__ len) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d >= n || ust[d] == ST_OK) return;
  status[d] = ust[d]; len[d] = 0;
}

// public V2 -> V1: per-document lengths from the scanned offsets
__global__ __launch_bounds__(256) void k_v2_lens(const uint64_t* __restrict__ off, const int32_t* __restrict__ st, uint32_t n,
                                                uint64_t* __restrict__ len) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d < n) len[d] = st[d] == ST_OK ? off[d + 1] - off[d] : 0u;
}

}  // namespace ygm

using namespace ygm;

extern "C" {

static int v2_rc(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { fprintf(stderr, "ygm: %s: %s\n", fn, hipGetErrorString(e)); return -1; }
  return 0;
}
size_t ygm_k_v2_cols() { return v2::C_N; }
int ygm_k_launch_v21(int pass, const uint8_t* arena, const uint64_t* upd_off, uint32_t n_upd, const uint32_t* doc_upd, uint32_t n_docs,
                     uint32_t mode, uint32_t flags, uint64_t* len_or_off, int32_t* st, uint8_t* out, uint8_t* cl, hipStream_t s) {
  if (n_upd == 0) return 0;
  const uint32_t g = (n_upd + V2_NT - 1) / V2_NT;
  if (pass == 0) {
    if (cl) hipLaunchKernelGGL(k_v21f<false>, dim3(g), dim3(V2_NT), 0, s, arena, upd_off, n_upd, doc_upd, n_docs, mode, len_or_off, st, cl, out);
    hipLaunchKernelGGL(k_v21_count, dim3(g), dim3(V2_NT), 0, s, arena, upd_off, n_upd, doc_upd, n_docs, mode, flags, len_or_off, st,
                       (const uint8_t*)cl);
  } else {
    if (cl) hipLaunchKernelGGL(k_v21f<true>, dim3(g), dim3(V2_NT), 0, s, arena, upd_off, n_upd, doc_upd, n_docs, mode, len_or_off, st, cl, out);
    hipLaunchKernelGGL(k_v21_write, dim3(g), dim3(V2_NT), 0, s, arena, upd_off, n_upd, mode, flags, (const uint64_t*)len_or_off,
                       (const int32_t*)st, out, (const uint8_t*)cl);
  }
  return v2_rc(__func__);
}
int ygm_k_launch_v12_count(const uint8_t* v1, const uint64_t* v1_off, const uint64_t* v1_len, const int32_t* v1_st, const uint8_t* v2a,
                           uint64_t v2n, const uint64_t* upd_off, const uint32_t* doc_upd, const int32_t* ust, uint32_t n_docs, uint32_t mode,
                           uint32_t flags, uint32_t* L, uint64_t* tot, int32_t* st, const uint8_t* claim, hipStream_t s) {
  if (n_docs == 0) return 0;
  const uint32_t g = (n_docs + V2_NT - 1) / V2_NT;
  hipLaunchKernelGGL(k_v12_count, dim3(g), dim3(V2_NT), 0, s, v1, v1_off, v1_len, v1_st, v2a, v2n, upd_off, doc_upd, ust, n_docs, mode, flags,
                     L, tot, st, claim);
  return v2_rc(__func__);
}
size_t ygm_k_v12_fast_scratch() {
  const size_t a = v12f_scratch<V12F_D, V12F_FS>(), b = v12f_scratch<2, (int)v2f::F_IN>();
  return a > b ? a : b;
}
int ygm_k_launch_v12_fast(const uint8_t* v1, const uint64_t* v1_off, const uint64_t* v1_len, const int32_t* v1_st, const uint64_t* slot_off,
                          const uint32_t* doc_upd, const int32_t* ust, uint32_t n_docs, uint8_t* out, uint64_t* fo, uint64_t* olen, int32_t* ost,
                          uint8_t* claim, unsigned long long* payload, uint8_t* scr, uint64_t slot_total, hipStream_t s) {
  if (n_docs == 0) return 0;
  // the grids of THIS device (the scratch was sized from the same calls, ygm_k_v12_fast_scratch)
  const uint32_t g1 = v12f_grid<V12F_D, V12F_FS>(), g2 = v12f_grid<2, (int)v2f::F_IN>();
  const uint32_t n1 = (n_docs + V12F_D - 1) / V12F_D, n2 = (n_docs + 1) / 2;
  hipLaunchKernelGGL((k_v12_fast<V12F_D, V12F_FS>), dim3(n1 < g1 ? n1 : g1), dim3(WAVE), 0, s, v1, v1_off, v1_len, v1_st, slot_off, doc_upd,
                     ust, n_docs, out, fo, olen, ost, claim, payload, 0, scr, slot_total);
  hipLaunchKernelGGL((k_v12_fast<2, (int)v2f::F_IN>), dim3(n2 < g2 ? n2 : g2), dim3(WAVE), 0, s, v1, v1_off, v1_len, v1_st, slot_off, doc_upd,
                     ust, n_docs, out, fo, olen, ost, claim, payload, 1, scr, slot_total);
  return v2_rc(__func__);
}
int ygm_k_launch_v12_write(const uint8_t* v1, const uint64_t* v1_off, const uint64_t* v1_len, const uint8_t* v2a, uint64_t v2n,
                           const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, uint32_t mode, uint32_t flags, const uint32_t* L,
                           const uint64_t* off, int32_t* st, uint8_t* out, uint64_t* out_len, const uint8_t* claim, uint64_t base, uint64_t* fo,
                           hipStream_t s) {
  if (n_docs == 0) return 0;
  const uint32_t g = (n_docs + V2_NT - 1) / V2_NT;
  hipLaunchKernelGGL(k_v12_write, dim3(g), dim3(V2_NT), 0, s, v1, v1_off, v1_len, v2a, v2n, upd_off, doc_upd, n_docs, mode, flags, L, off, st,
                     out, out_len, claim, base, fo);
  return v2_rc(__func__);
}
int ygm_k_launch_v2_status(const int32_t* ust, uint32_t n, int32_t* status, uint64_t* len, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_v2_status, dim3((n + 255) / 256), dim3(256), 0, s, ust, n, status, len);
  return v2_rc(__func__);
}

int ygm_k_launch_v2_lens(const uint64_t* off, const int32_t* st, uint32_t n, uint64_t* len, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_v2_lens, dim3((n + 255) / 256), dim3(256), 0, s, off, st, n, len);
  return v2_rc(__func__);
}

}  // extern "C"
