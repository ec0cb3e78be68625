// Development harness (tooling, never shipped): the flat-text snapshot (ygm_snap_text.hpp, k_snap_text's code)
// host-compiled beside the general one (ygm_snapshot.hpp) on a file of updates (snapdev's format).  For every
// document the text path takes, its bytes must equal the general path's.  Output: one line per document,
// "<taken 0/1> <general status> <equal 0/1>"; with out.bin, the text path's results in snapdev's format (status -1:
// not taken).
//     snaptext in.bin [flags] [budget] [out.bin]   (budget: LDS bytes of the workspace; default 6144)
#define YGM_HOST_BUILD 1
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../hocuspocus_amd/csrc/ygm_snap_text.hpp"

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: snaptext in.bin [flags] [budget]\n"); return 2; }
  const uint32_t flags = argc > 2 ? (uint32_t)atoi(argv[2]) : 0u;
  const uint32_t budget = argc > 3 ? (uint32_t)atoi(argv[3]) : 6144u;
  FILE* f = fopen(argv[1], "rb");
  FILE* g = argc > 4 ? fopen(argv[4], "wb") : nullptr;
  uint32_t n = 0; if (fread(&n, 4, 1, f) != 1) return 1;
  std::vector<uint8_t> ws, tws(budget + 64);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t len; if (fread(&len, 4, 1, f) != 1) return 1;
    std::vector<uint8_t> u(len + 64, 0);
    if (len && fread(u.data(), 1, len, f) != len) return 1;
    uint32_t S, D, C; ygm::snap::count_doc(u.data(), len, flags, S, D, C);
    const ygm::snap::Caps k = ygm::snap::caps_of(S, D, C, len);
    ws.assign(ygm::snap::ws_bytes(k) + 64, 0);
    uint32_t oo = 0, ol = 0;
    const int st = len ? ygm::snap::snapshot_doc(u.data(), len, flags, ws.data(), k, oo, ol) : 1;
    // the kernel's budget: the workspace (the input is read in place)
    const uint32_t sb = 0;
    bool taken = false, eq = false;
    if (len) {
      std::vector<uint8_t> out(2u * len + 48u, 0);
      ygm::snap::OutCap o{out.data(), 0, 2u * len + 48u};
      memset(tws.data(), 0xA5, tws.size());
      taken = ygm::snapt::snapshot_text(u.data(), len, flags, tws.data(), budget - sb, o) && o.n <= o.cap;
      if (taken) eq = st == 0 && o.n == ol && memcmp(out.data(), ws.data() + oo, ol) == 0;
      if (g) { const int32_t s32 = taken ? 0 : -1; const uint32_t l32 = taken ? o.n : 0u; fwrite(&s32, 4, 1, g); fwrite(&l32, 4, 1, g); if (l32) fwrite(out.data(), 1, l32, g); }
    } else if (g) { const int32_t s32 = -1; const uint32_t l32 = 0; fwrite(&s32, 4, 1, g); fwrite(&l32, 4, 1, g); }
    printf("%d %d %d\n", taken ? 1 : 0, st, eq ? 1 : 0);
  }
  fclose(f);
  if (g) fclose(g);
  return 0;
}
