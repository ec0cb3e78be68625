// fetch_cal.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access shapes of this engine's
// kernels (MI355X_MICROARCH.md §HBM: FETCH_SIZE is calibrated only for wide coalesced streaming reads, where it
// reports half the bytes; "other access widths are uncalibrated: calibrate on a known byte count in your own
// access pattern").  Each kernel reads a known number of bytes once, from a 2 GiB buffer (past the 256 MiB
// Infinity Cache); run it under `rocprofv3 --pmc FETCH_SIZE` and divide FETCH_SIZE by the printed bytes.
//
//   k_coal      wave-coalesced: lane i reads 16 B at base + 16 i, the wave walks 1 KiB per instruction
//   k_lane64    lane-per-stream in 64-byte chunks (the walker's staging, ygm_doc_walk.hpp): lane l owns a
//               contiguous region of `per` bytes and reads it as 4 x 16-byte loads per chunk
//   k_lane128   the same in 128-byte chunks (8 x 16-byte loads: whole lines)
//   k_wst       wave-coalesced 16-byte stores (WRITE_SIZE reference)
//   k_lst16     lane-per-stream 16-byte stores (the walker's output stores)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_cal tools/fetch_cal.hip   (tools/Makefile: fetch_cal)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_coal(const u32x4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) acc ^= p[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = 1;
}
template <int CH>   // chunk bytes per step: 64 or 128
__global__ __launch_bounds__(64) void k_lane(const uint8_t* __restrict__ p, uint64_t per, uint32_t* __restrict__ sink) {
  const uint64_t lane = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  const u32x4* s = (const u32x4*)(p + lane * per);
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t c = 0; c < per / CH; c++) {
#pragma unroll
    for (int j = 0; j < CH / 16; j++) acc ^= s[c * (CH / 16) + j];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = 1;
}
__global__ __launch_bounds__(256) void k_wst(u32x4* __restrict__ p, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) p[i] = u32x4{(uint32_t)i, 1, 2, 3};
}
__global__ __launch_bounds__(64) void k_lst16(uint8_t* __restrict__ p, uint64_t per) {
  const uint64_t lane = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  u32x4* s = (u32x4*)(p + lane * per);
  for (uint64_t c = 0; c < per / 16; c++) s[c] = u32x4{(uint32_t)c, 1, 2, 3};
}

int main() {
  const uint64_t bytes = 2ull << 30;
  uint8_t* p = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) { fprintf(stderr, "alloc failed\n"); return 1; }
  hipMemset(p, 1, bytes);
  hipDeviceSynchronize();
  const uint64_t per = 4096, lanes = bytes / per;   // 524 288 lane streams of 4 KiB (the C4 document size)
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_coal, dim3(8192), dim3(256), 0, 0, (const u32x4*)p, bytes / 16, sink);
    hipLaunchKernelGGL(k_lane<64>, dim3(lanes / 64), dim3(64), 0, 0, p, per, sink);
    hipLaunchKernelGGL(k_lane<128>, dim3(lanes / 64), dim3(64), 0, 0, p, per, sink);
    hipLaunchKernelGGL(k_wst, dim3(8192), dim3(256), 0, 0, (u32x4*)p, bytes / 16);
    hipLaunchKernelGGL(k_lst16, dim3(lanes / 64), dim3(64), 0, 0, p, per);
  }
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
  printf("{\"bytes_per_dispatch\": %llu, \"kernels\": [\"k_coal\", \"k_lane<64>\", \"k_lane<128>\", \"k_wst\", \"k_lst16\"], \"reps\": 2}\n",
         (unsigned long long)bytes);
  hipFree(p); hipFree(sink);
  return 0;
}
