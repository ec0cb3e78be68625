"""Host-API probe (tooling): ygm_merge_v1 (host arrays: chunks over two stage contexts, PCIe both ways) on a corpus,
wall / H2D / D2H / device time per call; the chunk size from YGM_CHUNK_MB (the engine reads it per call).

    python tools/host_probe.py c2|c3|c5 MB [MB ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from hocuspocus_amd import Engine
    from tools import synth
    kind, mbs = sys.argv[1], sys.argv[2:]
    if kind == "c2":
        arena, upd_off, doc_upd = synth.text_updates(100000, 200, 1, 4, seed=3)
    elif kind == "c3":
        arena, upd_off, doc_upd = synth.big_docs(100000, 10_000_000, 1024, max_clients=64, max_k=200, seed=8)
    else:
        arena, upd_off, doc_upd = synth.big_docs(1000, 1_000_000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
    n = len(doc_upd) - 1
    upd_doc = np.repeat(np.arange(n, dtype=np.uint32), np.diff(doc_upd.astype(np.int64)))
    e = Engine(0)
    for mb in mbs:
        os.environ["YGM_CHUNK_MB"] = mb
        e.merge_packed_raw(arena, upd_off, upd_doc, n)
        s0 = e.stats()
        t0 = time.perf_counter()
        for _ in range(3):
            e.merge_packed_raw(arena, upd_off, upd_doc, n)
        wall = (time.perf_counter() - t0) / 3
        s1 = e.stats()
        print(json.dumps({"corpus": kind, "chunk_mb": int(mb), "wall_ms": round(wall * 1e3, 2),
                          "h2d_ms": round((s1.h2d_ms - s0.h2d_ms) / 3, 2), "d2h_ms": round((s1.d2h_ms - s0.d2h_ms) / 3, 2),
                          "device_ms": round((s1.kernel_ms - s0.kernel_ms) / 3, 2)}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
