// Host build of the device V2 transcoders (hocuspocus_amd/csrc/ygm_v2.hpp) for development on a machine
// without a GPU: tools/v2dev/check.py drives them around the CPU oracle's V1 functions over the golden
// vectors.  Development tooling only; never loaded by the product or the tests.
#define YGM_HOST_BUILD 1
#include <stdint.h>
#include <string.h>
#include <math.h>
#include "../../hocuspocus_amd/csrc/ygm_v2.hpp"

using namespace ygm;

extern "C" {
// V2 -> V1 of one update at arena[off, off + n); out == nullptr: size only
int hv_v21(const uint8_t* arena, uint64_t off, uint32_t n, uint32_t mode, uint32_t flags, uint8_t* out, uint64_t* out_len) {
  Out o{out, 0};
  const int e = v2::v21(arena + off, n, off, mode, flags, o);
  *out_len = o.n;
  return e;
}
// V1 -> V2 of one update (count pass, then the write pass when out != nullptr)
int hv_v12(const uint8_t* v1, uint32_t n, const uint8_t* v2a, uint64_t v2n, uint32_t mode, uint32_t flags, uint8_t* out, uint64_t* out_len) {
  v2::Enc2 w; v2::enc_init(w);
  int e = v2::v12_body(v1, n, v2a, v2n, mode, flags, w);
  if (e) { *out_len = 0; return e; }
  uint32_t L[v2::C_N];
  for (int i = 0; i < v2::C_N; i++) L[i] = w.o[i].n;
  *out_len = v2::v2_total(L);
  if (!out) return 0;
  return v2::v12_write(v1, n, v2a, v2n, mode, flags, L, out);
}
}

#include "../../hocuspocus_amd/csrc/ygm_v2_fast.hpp"
extern "C" {
// the register-resident fast V1 -> V2 encoder (ygm_v2_fast.hpp) over a staged copy of v1 (zero slack past n):
// 0 = done (out gets the V2 bytes), 1 = off the fast path, 2 = past the fast path's sizes
int hv_v12f(const uint8_t* v1, uint32_t n, uint8_t* out, uint64_t* out_len) {
  *out_len = 0;
  if (n > v2f::F_IN) return 2;
  static uint8_t in[v2f::F_IN + 128], ob[v2f::F_OUT + 64];
  static uint64_t m[(v2f::F_IN + 128) / 64 + 2];
  memset(in, 0, sizeof in); memcpy(in, v1, n);
  for (uint32_t k = 0; k < (v2f::F_IN + 128) / 64; k++) m[k] = v2f::f_mask_word((const uint8_t*)in, k);
  const v2f::FSrc<const uint8_t*, const uint64_t*> src{in, m};
  // the kernel's nine lanes, one after the other: count passes, layout, write passes
  uint32_t L[v2f::FC_N], base[v2f::FC_N];
  v2f::FCS c;
  for (uint32_t col = 0; col < v2f::FC_N; col++) {
    if (!v2f::f_col_run(src, 0u, n, col, (uint8_t*)nullptr, 0u, 0u, c)) return 1;
    L[col] = c.n;
  }
  const uint32_t t = v2f::fc_layout((uint8_t*)nullptr, L, base);
  if (t > v2f::F_OUT) return 2;
  (void)v2f::fc_layout(ob, L, base);
  for (uint32_t col = 0; col < v2f::FC_N; col++)
    if (!v2f::f_col_run(src, 0u, n, col, ob, base[col], 0xFFFFFFFFu, c)) return 3;   // (cannot happen: the count pass took the same path)
  memcpy(out, ob, t);
  *out_len = t;
  return 0;
}
}

#include "../../hocuspocus_amd/csrc/ygm_v21_fast.hpp"
extern "C" {
// the register-resident fast V2 -> V1 transcoder (ygm_v21_fast.hpp, the k_v21_* kernels' first try): 0 = done (size
// pass, then the bytes when out != nullptr), 1 = off the fast path
int hv_v21f(const uint8_t* u, uint32_t n, uint32_t mode, uint8_t* out, uint64_t* out_len) {
  const v21f::Src<const uint8_t*> s{u};
  v21f::BOut<uint8_t*> c{nullptr, 0};
  *out_len = 0;
  if (!v21f::v21_fast(s, n, mode, c)) return 1;
  *out_len = c.n;
  if (!out) return 0;
  v21f::BOut<uint8_t*> o{out, 0};
  if (!v21f::v21_fast(s, n, mode, o) || o.n != c.n) return 3;
  return 0;
}
}
