// Dev microbenchmark (tooling): 64 streams per wave (one per "document", S bytes each), each advancing
// 16*P bytes per round through P load instructions; G lanes share each 16*G-byte run of one stream
// (G = 1: every lane reads its own stream, the ring walker's shape).   ./ldbench n_streams S waves_per_cu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%d %s\n", __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
template <int G, int P>
__global__ __launch_bounds__(64) void k_rd(const u4* __restrict__ a, uint32_t S, uint32_t nstreams, unsigned* __restrict__ sink) {
  const uint32_t l = threadIdx.x;
  unsigned acc = 0;
  for (uint32_t s0 = blockIdx.x * 64; s0 < nstreams; s0 += gridDim.x * 64) {
    for (uint32_t off = 0; off + 16 * P <= S; off += 16 * P) {
      u4 r[P];
#pragma unroll
      for (int j = 0; j < P; j++) {
        const uint32_t stream = s0 + (64 / G) * (j % G) + l / G;
        const uint32_t piece = off / 16 + G * (j / G) + (l % G);
        r[j] = a[(uint64_t)stream * (S / 16) + piece];
      }
#pragma unroll
      for (int j = 0; j < P; j++) acc ^= r[j].x + r[j].y + r[j].z + r[j].w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
int main(int argc, char** argv) {
  const uint32_t ns = argc > 1 ? atoi(argv[1]) : 1000000, S = argc > 2 ? atoi(argv[2]) : 3328, wpc = argc > 3 ? atoi(argv[3]) : 8;
  const uint64_t bytes = (uint64_t)ns * S;
  void* a; unsigned* sink;
  CK(hipMalloc(&a, bytes + 4096)); CK(hipMalloc(&sink, 64)); CK(hipMemset(a, 1, bytes));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t grid = prop.multiProcessorCount * wpc;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int Gs[6] = {1, 2, 4, 1, 4, 8}, Ps[6] = {4, 4, 4, 8, 8, 8};
  for (int g = 0; g < 6; g++) {
    float best = 1e9;
    for (int r = 0; r < 4; r++) {
      CK(hipEventRecord(e0));
      switch (g) {
        case 0: hipLaunchKernelGGL((k_rd<1, 4>), dim3(grid), dim3(64), 0, 0, (const u4*)a, S, ns, sink); break;
        case 1: hipLaunchKernelGGL((k_rd<2, 4>), dim3(grid), dim3(64), 0, 0, (const u4*)a, S, ns, sink); break;
        case 2: hipLaunchKernelGGL((k_rd<4, 4>), dim3(grid), dim3(64), 0, 0, (const u4*)a, S, ns, sink); break;
        case 3: hipLaunchKernelGGL((k_rd<1, 8>), dim3(grid), dim3(64), 0, 0, (const u4*)a, S, ns, sink); break;
        case 4: hipLaunchKernelGGL((k_rd<4, 8>), dim3(grid), dim3(64), 0, 0, (const u4*)a, S, ns, sink); break;
        case 5: hipLaunchKernelGGL((k_rd<8, 8>), dim3(grid), dim3(64), 0, 0, (const u4*)a, S, ns, sink); break;
      }
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    printf("{\"G\": %d, \"P\": %d, \"wpc\": %u, \"ms\": %.3f, \"GBps\": %.0f}\n", Gs[g], Ps[g], wpc, best, bytes / best / 1e6);
  }
  return 0;
}
