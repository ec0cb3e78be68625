// Development harness (tooling, never shipped): runs the device snapshot code (ygm_snapshot.hpp) on the
// host over a file of updates, so the kernel's logic can be iterated against the yjs bundle in the
// build container.  Input: u32 count, then (u32 len, bytes) per update.  Output: (i32 status, u32 len,
// bytes) per update; a document left pending (status 64) writes its PendHdr and three updates.
#define YGM_HOST_BUILD 1
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../hocuspocus_amd/csrc/ygm_snapshot.hpp"

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: snapdev in.bin out.bin [flags]\n"); return 2; }
  const uint32_t flags = argc > 3 ? (uint32_t)atoi(argv[3]) : 0u;
  FILE* f = fopen(argv[1], "rb"); FILE* g = fopen(argv[2], "wb");
  uint32_t n = 0; if (fread(&n, 4, 1, f) != 1) return 1;
  std::vector<uint8_t> ws;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t len; if (fread(&len, 4, 1, f) != 1) return 1;
    std::vector<uint8_t> u(len + 64, 0);
    if (len && fread(u.data(), 1, len, f) != len) return 1;
    uint32_t S, D, C; ygm::snap::count_doc(u.data(), len, flags, S, D, C);
    const ygm::snap::Caps k = ygm::snap::caps_of(S, D, C, len);
    ws.assign(ygm::snap::ws_bytes(k) + 64, 0);
    uint32_t oo = 0, ol = 0;
    const int st = ygm::snap::snapshot_doc(u.data(), len, flags, ws.data(), k, oo, ol);
    const int32_t s32 = st; const uint32_t l32 = (st == 0 || st == ygm::snap::ST_PEND) ? ol : 0u;   // (ST_PEND: PendHdr + three updates)
    fwrite(&s32, 4, 1, g); fwrite(&l32, 4, 1, g);
    if (l32) fwrite(ws.data() + oo, 1, l32, g);
  }
  fclose(f); fclose(g);
  return 0;
}
