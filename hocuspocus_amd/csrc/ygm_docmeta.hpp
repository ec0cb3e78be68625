// ygm_docmeta.hpp -- what the kernel files share: the per-launch device counters, merge output slots, and the
// launch glue's device-size cache and error report.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <atomic>

#include "ygm_common.hpp"

namespace ygm {

struct DocMeta {                    // per-launch device counters (zeroed by the launcher)
  unsigned int ticket;
  unsigned int fault;
  unsigned int fb_count;            // documents sent to the sequential kernel
  unsigned int defer_count;         // documents sent from the wave kernel to the workgroup kernel
  unsigned int lean_defer;          // documents sent from the lean kernel to the wave kernel
  unsigned int big_defer;           // documents sent from the large-document kernel to the sequential kernel
  unsigned int wide_defer;          // documents sent from the wide lean kernel to the wave kernel
  unsigned int mid_defer;           // documents sent from the mid-size large-document kernel to the large size
  unsigned int big_started;         // 16-wave large-document workgroups started (k_big_wait)
  unsigned int route_n;           // documents the big-tier routing pass leaves to the wave kernel
  unsigned long long big_scur;      // large-document kernel: struct-record entries carved
  unsigned long long fast_total;    // SV/diff: bytes of the packed (look-back placed) output
  unsigned long long cursor;        // merge: bytes in the overflow region (after the per-document slots)
  unsigned long long payload;       // merge: sum of output lengths (algorithmic output bytes)
  unsigned long long fb_upds;       // updates / bytes of fallback documents (scratch sizing)
  unsigned long long fb_bytes;
  unsigned long long scr_upd_cursor;
  unsigned long long scr_byte_cursor;
  unsigned long long big_cursor;      // large-document kernel: block-table entries carved (16-byte multiple:
                                      // the lean kernel zeroes slots in 16-byte pieces)
  unsigned long long payload_sh[16 * 16]; // merge: output lengths summed in 16 shards, one 128-B line each (no hot atomic line)
};
YDEV void add_payload(DocMeta* m, uint32_t d, uint64_t n) { atomicAdd(&m->payload_sh[(d & 15u) * 16u], (unsigned long long)n); }

// Merge output placement.  Document d owns the 16-byte aligned slot starting at
// align16(2*b0 + 64d) with capacity 2*(b1-b0) + 48 (b0, b1 = its input byte
// range), inside [2*b0 + 64d, 2*b1 + 64(d+1)): slots never overlap and need no
// cross-document scan (slot_total = 2*arena + 64*n_docs).  An output that does
// not fit its slot goes to the overflow region after slot_total (atomic cursor).
YDEV uint64_t merge_slot(uint64_t b0, uint32_t d) { return (2 * b0 + 64ull * d + 15) & ~15ull; }
YDEV uint64_t merge_slot_cap(uint64_t nbytes) { return 2 * nbytes + 48; }
YDEV uint64_t dw_shfl64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src);
  return ((uint64_t)hi << 32) | lo;
}

// ======================================================================= launch glue
// a failed launch names its kernel and the HIP error on stderr (the C ABI only returns YGM_EDEVICE)
// persistent grid sizes are cached per device: a pool may drive GPUs of different sizes, its contexts from
// different threads (the first computation on each device wins; a racing second one stores the same value)
constexpr int YGM_MAX_DEVICES = 64;
template <class F>
static uint32_t per_device(std::atomic<uint32_t> (&cache)[YGM_MAX_DEVICES], F compute) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::atomic<uint32_t>& slot = cache[(unsigned)dev % YGM_MAX_DEVICES];
  uint32_t v = slot.load(std::memory_order_relaxed);
  if (!v) { v = compute(); slot.store(v, std::memory_order_relaxed); }
  return v;
}
static uint32_t device_cus() {
  static std::atomic<uint32_t> cache[YGM_MAX_DEVICES];
  return per_device(cache, [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? (uint32_t)n : 256u;
  });
}

static int launch_rc(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fprintf(stderr, "ygm: %s: %s\n", fn, hipGetErrorString(e));
  return (int)e;
}

}  // namespace ygm
