// ygm_common.hpp -- workgroup / wave primitives for the ygm kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ygm_v1.hpp"

namespace ygm {

constexpr int WAVE = 64;

YDEV uint32_t lane_id() { return __lane_id(); }

template <class T>
YDEV T wave_incl_scan_add(T v) {
  const int l = (int)lane_id();
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const T o = __shfl_up(v, d, WAVE);
    if (l >= d) v += o;
  }
  return v;
}
template <class T>
YDEV T wave_incl_scan_max(T v) {
  const int l = (int)lane_id();
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const T o = __shfl_up(v, d, WAVE);
    if (l >= d && o > v) v = o;
  }
  return v;
}
template <class T>
YDEV T wave_sum(T v) {
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, WAVE);
  return v;
}

// Block-wide exclusive scan of one value per thread; returns prefix, sets *total.
// `tmp` must hold NT/64 + 1 entries of T in LDS.  Contains barriers.
template <int NT, class T>
YDEV T block_exscan(T v, T* tmp, T& total) {
  const int t = threadIdx.x, w = t / WAVE, l = t % WAVE;
  const T inc = wave_incl_scan_add(v);
  if (l == WAVE - 1) tmp[w] = inc;
  __syncthreads();
  if (t == 0) {
    T run = 0;
    for (int i = 0; i < NT / WAVE; i++) { const T x = tmp[i]; tmp[i] = run; run += x; }
    tmp[NT / WAVE] = run;
  }
  __syncthreads();
  const T r = tmp[w] + inc - v;
  total = tmp[NT / WAVE];
  __syncthreads();
  return r;
}

// In-place exclusive scan of a[0..n) by NT threads (contiguous chunks per thread).
// Returns the total.  Contains barriers.
template <int NT, class T>
YDEV T block_scan_array(T* a, int n, T* tmp) {
  const int t = threadIdx.x;
  const int per = (n + NT - 1) / NT;
  const int b = t * per, e = min(n, b + per);
  T s = 0;
  for (int i = b; i < e; i++) s += a[i];
  T total;
  T run = block_exscan<NT>(s, tmp, total);
  for (int i = b; i < e; i++) { const T x = a[i]; a[i] = run; run += x; }
  __syncthreads();
  return total;
}
// In-place inclusive max-scan of a[0..n).
template <int NT, class T>
YDEV void block_maxscan_array(T* a, int n, T* tmp, T lowest) {
  const int t = threadIdx.x, w = t / WAVE, l = t % WAVE;
  const int per = (n + NT - 1) / NT;
  const int b = t * per, e = min(n, b + per);
  T m = lowest;
  for (int i = b; i < e; i++) m = a[i] > m ? a[i] : m;
  // exclusive max over threads
  T inc = wave_incl_scan_max(m);
  if (l == WAVE - 1) tmp[w] = inc;
  __syncthreads();
  if (t == 0) {
    T run = lowest;
    for (int i = 0; i < NT / WAVE; i++) { const T x = tmp[i]; tmp[i] = run; run = x > run ? x : run; }
  }
  __syncthreads();
  T ex = __shfl_up(inc, 1, WAVE);
  if (l == 0) ex = lowest;
  T run = tmp[w] > ex ? tmp[w] : ex;
  for (int i = b; i < e; i++) { run = a[i] > run ? a[i] : run; a[i] = run; }
  __syncthreads();
}

// Bitonic sort of (key, val) pairs in LDS; n is a power of two.  Contains barriers.
template <int NT, class K, class V>
YDEV void bitonic_sort(K* key, V* val, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n / 2; i += NT) {
        const int lo = ((i / j) * 2 * j) + (i % j);
        const int hi = lo + j;
        const bool up = (lo & k) == 0;
        const K a = key[lo], b = key[hi];
        if ((a > b) == up) { key[lo] = b; key[hi] = a; const V t = val[lo]; val[lo] = val[hi]; val[hi] = t; }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- look-back
// Decoupled look-back over tiles taken in ticket order (tile t only waits on
// tiles < t, which started earlier, so progress is guaranteed).  Each status
// word is ONE 8-byte {flag:2 | value:62} granule written by one agent-scope
// atomic store and read by agent-scope atomic loads (MI355X_MICROARCH.md
// "Valid forms": the data IS the flag; no fences needed).  Spins are bounded:
// on timeout *fault is set and the caller marks its documents YGM_EDEVICE.
constexpr uint64_t LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1;

YDEV void lb_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
YDEV unsigned long long lb_load(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Must be called by ALL 64 lanes of exactly one wave.  Returns the exclusive prefix.
YDEV uint64_t lookback(unsigned long long* st, uint32_t tile, uint64_t agg, unsigned int* fault) {
  const int l = (int)lane_id();
  if (tile == 0) {
    if (l == 0) lb_store(&st[0], LB_INC | agg);
    return 0;
  }
  if (l == 0) lb_store(&st[tile], LB_AGG | agg);
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  uint32_t spins = 0;
  for (;;) {
    const int64_t idx = base - l;
    const unsigned long long w = idx >= 0 ? lb_load(&st[idx]) : LB_INC;
    const uint32_t flag = (uint32_t)(w >> 62);
    const unsigned long long incl = __ballot(flag == 2);
    const unsigned long long nready = __ballot(flag == 0);
    const int first = incl ? __ffsll((long long)incl) - 1 : WAVE;
    const unsigned long long need = first >= WAVE - 1 ? ~0ull : ((2ull << first) - 1);
    if (nready & need) {
      if (++spins > (1u << 22)) { if (l == 0) atomicOr(fault, 1u); return 0; }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint64_t v = (l <= first) ? (uint64_t)(w & LB_VAL) : 0;
    excl += wave_sum(v);
    if (first < WAVE) break;
    base -= WAVE;
  }
  if (l == 0) lb_store(&st[tile], LB_INC | (excl + agg));
  return excl;
}

}  // namespace ygm
