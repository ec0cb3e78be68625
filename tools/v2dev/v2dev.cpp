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
