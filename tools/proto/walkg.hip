// Dev harness (tooling, not product): times the register-window walker (ygm_walk_g.hpp) on a C4 corpus
// and checks every document against the CPU oracle.   ./walkg n_docs waves_per_cu [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../../hocuspocus_amd/csrc/ygm_doc_walk.hpp"
namespace ygm {
YDEV uint64_t merge_slot(uint64_t b0, uint32_t d) { return (2 * b0 + 64ull * d + 15) & ~15ull; }
YDEV uint64_t merge_slot_cap(uint64_t nbytes) { return 2 * nbytes + 48; }
YDEV uint64_t dw_shfl64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src);
  return ((uint64_t)hi << 32) | lo;
}
}
#include "ygm_walk_g.hpp"
extern "C" {
void *synth_text_states_gen(uint64_t seed, const uint32_t *idx, uint32_t n_docs, uint32_t min_bytes, uint32_t max_bytes,
                            uint32_t min_clients, uint32_t max_clients, uint32_t threads, uint64_t *out_bytes, uint64_t *out_sv_bytes);
void synth_text_states_take(void *h, uint8_t *buf, uint64_t *doc_off, uint8_t *sv, uint64_t *sv_off);
int yo_sv(const uint8_t *u, size_t ulen, int flags, uint8_t **out, size_t *out_len);
int yo_diff(const uint8_t *u, size_t ulen, const uint8_t *sv, size_t svlen, int flags, uint8_t **out, size_t *out_len);
void yo_free(void *p);
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? atoi(argv[1]) : 100000, wpc = argc > 2 ? atoi(argv[2]) : 16, reps = argc > 3 ? atoi(argv[3]) : 5;
  uint64_t nb, ns;
  void *h = synth_text_states_gen(3, nullptr, n, 1024, 8192, 1, 16, 16, &nb, &ns);
  std::vector<uint8_t> arena(nb + 64, 0), sv(ns + 64, 0);
  std::vector<uint64_t> doff(n + 1), soff(n + 1);
  synth_text_states_take(h, arena.data(), doff.data(), sv.data(), soff.data());
  uint8_t *d_a, *d_out; uint64_t *d_off, *d_oo, *d_ol; int32_t *d_st; unsigned *d_dc; uint32_t *d_dl; unsigned long long *d_pay;
  const uint64_t cap = 2 * nb + 64ull * n + 4096;
  CK(hipMalloc(&d_a, nb + 64)); CK(hipMalloc(&d_out, cap)); CK(hipMalloc(&d_off, 8 * (n + 1)));
  CK(hipMalloc(&d_oo, 8 * n)); CK(hipMalloc(&d_ol, 8 * n)); CK(hipMalloc(&d_st, 4 * n)); CK(hipMalloc(&d_dc, 4));
  CK(hipMalloc(&d_dl, 4 * n)); CK(hipMalloc(&d_pay, 8));
  CK(hipMemcpy(d_a, arena.data(), nb + 64, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_off, doff.data(), 8 * (n + 1), hipMemcpyHostToDevice));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t grid = prop.multiProcessorCount * wpc;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e9; unsigned long long pay = 0; unsigned dc = 0;
  for (uint32_t r = 0; r < reps; r++) {
    CK(hipMemset(d_dc, 0, 4)); CK(hipMemset(d_pay, 0, 8)); CK(hipMemset(d_st, 0xFF, 4 * n));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(ygm::k_walk_g<0>, dim3(grid), dim3(64), 0, 0, d_a, d_off, n, d_out, d_oo, d_ol, d_st, d_dc, d_dl, cap, d_pay);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  CK(hipMemcpy(&pay, d_pay, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(&dc, d_dc, 4, hipMemcpyDeviceToHost));
  std::vector<uint64_t> oo(n), ol(n); std::vector<int32_t> st(n); std::vector<uint8_t> out(cap);
  CK(hipMemcpy(oo.data(), d_oo, 8 * n, hipMemcpyDeviceToHost)); CK(hipMemcpy(ol.data(), d_ol, 8 * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(st.data(), d_st, 4 * n, hipMemcpyDeviceToHost)); CK(hipMemcpy(out.data(), d_out, cap, hipMemcpyDeviceToHost));
  uint64_t bad = 0, fb = 0, okd = 0;
  for (uint32_t d = 0; d < n; d++) {
    if (st[d] == 100) { fb++; continue; }
    uint8_t *o; size_t ln;
    const int s = yo_sv(arena.data() + doff[d], doff[d + 1] - doff[d], 0, &o, &ln);
    if (s != st[d] || (s == 0 && (ln != ol[d] || memcmp(o, out.data() + oo[d], ln)))) { if (bad < 5) fprintf(stderr, "doc %u: st %d/%d len %zu/%lu\n", d, s, st[d], ln, (unsigned long)ol[d]); bad++; }
    else okd++;
    if (s == 0) yo_free(o);
  }
  const double algo = (double)nb + (double)pay;
  printf("{\"docs\": %u, \"waves_per_cu\": %u, \"best_ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f, \"ok\": %lu, \"fallback\": %lu, \"defer_cnt\": %u, \"mismatch\": %lu}\n",
         n, wpc, best, algo / best / 1e6, algo / best / 1e6 / 8000.0, (unsigned long)okd, (unsigned long)fb, dc, (unsigned long)bad);
  return bad ? 1 : 0;
}
