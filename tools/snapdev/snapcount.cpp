// Development harness (tooling, never shipped): the snapshot workspace's used counts per document (structs S,
// delete-set ranges D, client blocks C, items after splits, pieces, tx ranges, types, bytes) for sizing an
// LDS-resident workspace.  Input as snapdev (u32 count, then (u32 len, bytes) per update); one line per document.
#define YGM_HOST_BUILD 1
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../hocuspocus_amd/csrc/ygm_snapshot.hpp"

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: snapcount in.bin [flags]\n"); return 2; }
  const uint32_t flags = argc > 2 ? (uint32_t)atoi(argv[2]) : 0u;
  FILE* f = fopen(argv[1], "rb");
  uint32_t n = 0; if (fread(&n, 4, 1, f) != 1) return 1;
  std::vector<uint8_t> ws;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t len; if (fread(&len, 4, 1, f) != 1) return 1;
    std::vector<uint8_t> u(len + 64, 0);
    if (len && fread(u.data(), 1, len, f) != len) return 1;
    uint32_t S, D, C; ygm::snap::count_doc(u.data(), len, flags, S, D, C);
    const ygm::snap::Caps k = ygm::snap::caps_of(S, D, C, len);
    ws.assign(ygm::snap::ws_bytes(k) + 64, 0);
    ygm::snap::Doc d;
    uint8_t* p = ws.data();
    d.in = u.data(); d.n = len; d.flags = flags; d.err = 0; d.epoch = 0; d.n_ins = 0; d.hint_id = 0; d.hint_k = -1;
    d.it = (ygm::snap::SI*)p; d.n_it = 0; d.cap_it = k.it; p += ygm::snap::al16((uint64_t)k.it * sizeof(ygm::snap::SI));
    d.pc = (ygm::snap::Piece*)p; d.n_pc = 0; d.cap_pc = k.pc; p += ygm::snap::al16((uint64_t)k.pc * sizeof(ygm::snap::Piece));
    d.ty = (ygm::snap::TypeRec*)p; d.n_ty = 0; d.cap_ty = k.ty; p += ygm::snap::al16((uint64_t)k.ty * sizeof(ygm::snap::TypeRec));
    d.me = (ygm::snap::MapEnt*)p; d.n_me = 0; d.cap_me = k.me; p += ygm::snap::al16((uint64_t)k.me * sizeof(ygm::snap::MapEnt));
    d.cl = (ygm::snap::Cli*)p; d.n_cl = 0; d.cap_cl = k.cl; p += ygm::snap::al16((uint64_t)k.cl * sizeof(ygm::snap::Cli));
    d.tx = (ygm::snap::Rng*)p; d.n_tx = 0; d.cap_tx = k.tx; p += ygm::snap::al16((uint64_t)k.tx * sizeof(ygm::snap::Rng));
    d.dsin = (ygm::snap::Rng*)p; d.n_dsin = 0; d.cap_dsin = k.dsin; p += ygm::snap::al16((uint64_t)k.dsin * sizeof(ygm::snap::Rng));
    d.pds = (ygm::snap::Rng*)p; d.n_pds = 0; d.n_rest = 0; d.pend = false; p += ygm::snap::al16((uint64_t)k.dsin * sizeof(ygm::snap::Rng));
    d.st = (int32_t*)p; d.cap_st = k.st; p += ygm::snap::al16(4ull * k.st);
    d.seq = (int32_t*)p; d.cap_seq = k.seq; p += ygm::snap::al16(4ull * k.seq);
    d.ch = (int32_t*)p; d.ch_mask = k.hc - 1u; p += ygm::snap::al16(4ull * k.hc);
    d.out = p; d.cap_out = k.out;
    const uint32_t ol = d.run();
    printf("%d %u %u %u %u %u %u %u %u %u %u %u\n", d.err, len, S, D, C, d.n_it, d.n_pc, d.n_tx, d.n_ty, d.n_me, ol, d.epoch);
  }
  fclose(f);
  return 0;
}
