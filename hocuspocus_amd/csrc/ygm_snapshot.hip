// ygm_snapshot.hip -- doc-normalized snapshot kernels: one thread per document runs
// ygm_snapshot.hpp over a workspace carved from one device arena.
//   k_snap_count : per document, the struct / delete-range / client-block counts -> workspace bytes
//   k_snap_scan* : exclusive scan of the workspace sizes (three launches, 256 documents per block)
//   k_snap       : per document, integrate + gc + merge + encode into its workspace's output region
// A thread per document keeps the reference's sequential algorithm (YATA integration order matters)
// while 64 documents share a wave; the workspace is per document, so nothing is shared.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ygm_common.hpp"
#include "ygm_snapshot.hpp"

namespace ygm {

constexpr int SN_NT = 64;   // one wave per block: documents are independent

__global__ __launch_bounds__(SN_NT) void k_snap_count(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off,
                                                     uint32_t n_docs, uint32_t flags, uint4* __restrict__ cnt,
                                                     uint64_t* __restrict__ need) {
  const uint32_t d = blockIdx.x * SN_NT + threadIdx.x;
  if (d >= n_docs) return;
  const uint64_t a = doc_off[d], b = doc_off[d + 1];
  uint32_t S = 0, D = 0, C = 0;
  const uint32_t n = b > a && b - a < (1ull << 30) ? (uint32_t)(b - a) : 0u;
  if (n) snap::count_doc(arena + a, n, flags, S, D, C);
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
                                               int32_t* __restrict__ status, unsigned long long* __restrict__ payload, uint32_t dpw) {
  // dpw documents per wave (lanes >= dpw idle): the per-document code diverges from lane to lane, so
  // fewer documents per wave trade SIMD lanes for less serialised divergence and more waves in flight
  const uint32_t d = blockIdx.x * dpw + threadIdx.x;
  uint64_t mine = 0;
  if (threadIdx.x < dpw && d < n_docs) {
    const uint4 c = cnt[d];
    const uint64_t a = doc_off[d], b = doc_off[d + 1];
    int st = ST_OK;
    uint32_t oo = 0, ol = 0;
    if (b < a || b - a >= (1ull << 30)) st = ST_INVAL;
    else if (c.w == 0) st = ST_MALFORMED;   // (an empty update: yjs throws reading it)
    else {
      const snap::Caps k = snap::caps_of(c.x, c.y, c.z, c.w);
      st = snap::snapshot_doc(arena + a, c.w, flags, ws + ws_off[d], k, oo, ol);
    }
    out_off[d] = ws_off[d] + oo;
    out_len[d] = st == ST_OK ? ol : 0u;
    status[d] = st;
    mine = st == ST_OK ? ol : 0u;
  }
  mine = wave_sum(mine);
  if ((threadIdx.x & (WAVE - 1)) == 0 && mine) atomicAdd(payload, (unsigned long long)mine);
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
int ygm_k_launch_snap_plan(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, void* cnt, uint64_t* ws_off,
                           uint64_t* bs, hipStream_t s) {
  if (n_docs == 0) return 0;
  const uint32_t g = (n_docs + SN_NT - 1) / SN_NT, nb = (n_docs + 1 + 255) / 256;
  hipLaunchKernelGGL(k_snap_count, dim3(g), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, (uint4*)cnt, ws_off);
  hipLaunchKernelGGL(k_snap_scan_sum, dim3(nb), dim3(256), 0, s, (const uint64_t*)ws_off, n_docs, bs);
  hipLaunchKernelGGL(k_snap_scan_top, dim3(1), dim3(1024), 0, s, bs, nb);
  hipLaunchKernelGGL(k_snap_scan_apply, dim3(nb), dim3(256), 0, s, ws_off, n_docs, (const uint64_t*)bs);
  return snap_rc(__func__);
}
// phase 2: the snapshots (ws sized from ws_off[n_docs])
int ygm_k_launch_snap(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, const void* cnt, const uint64_t* ws_off,
                      uint8_t* ws, uint64_t* out_off, uint64_t* out_len, int32_t* status, unsigned long long* payload, hipStream_t s) {
  if (n_docs == 0) return 0;
  const char* env = getenv("YGM_SNAP_DPW");
  uint32_t dpw = env ? (uint32_t)atoi(env) : 4u;
  if (dpw < 1 || dpw > (uint32_t)SN_NT) dpw = 4u;
  const uint32_t g = (n_docs + dpw - 1) / dpw;
  hipLaunchKernelGGL(k_snap, dim3(g), dim3(SN_NT), 0, s, arena, doc_off, n_docs, flags, (const uint4*)cnt, ws_off, ws, out_off, out_len,
                     status, payload, dpw);
  return snap_rc(__func__);
}

}  // extern "C"
