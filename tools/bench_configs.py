"""Throughput probes for the non-headline configs (tooling; bench.py stays the C2 contract).

    python tools/bench_configs.py c4 [n_docs]     state vector + diffUpdate over synthetic merged states (C4)
    python tools/bench_configs.py c2del [n_docs]  C2 with 20 % deletes
    python tools/bench_configs.py c3 [n_docs] [max_bytes]   [snapshot, ...log] Zipf-sized documents (C3)
    python tools/bench_configs.py c5 [n_docs] [max_bytes]   XmlFragment documents over ~10k client blocks (C5)
Prints one JSON line per op: kernel ms, docs/s, algorithmic GB/s."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hocuspocus_amd import Engine  # noqa: E402
from tools import synth  # noqa: E402


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(torch.device("cuda", 0))


def c4(n):
    t0 = time.time()
    arena, doc_off, sva, sv_off = synth.text_states(n, seed=3)
    gen = time.time() - t0
    e = Engine(0)
    da = dev(np.concatenate([arena, np.zeros(64, np.uint8)]))
    do = dev(doc_off.view(np.int64))
    ds = dev(np.concatenate([sva, np.zeros(64, np.uint8)]))
    dso = dev(sv_off.view(np.int64))
    for op in ("sv", "diff"):
        for rep in range(4):
            s0 = e.stats()
            if op == "sv":
                r = e.sv_device(da.data_ptr(), len(arena), do.data_ptr(), n)
            else:
                r = e.diff_device(da.data_ptr(), len(arena), do.data_ptr(), ds.data_ptr(), dso.data_ptr(), n)
            s1 = e.stats()
        ms = s1.kernel_ms - s0.kernel_ms
        algo = len(arena) + r.payload_bytes + (len(sva) if op == "diff" else 0)
        print(json.dumps({"config": "C4", "op": op, "docs": n, "bytes_in": len(arena), "kernel_ms": round(ms, 3),
                          "walker_ms": round(s1.lean_ms - s0.lean_ms, 3), "walker_docs": s1.docs_lean - s0.docs_lean,
                          "exact_docs": s1.docs_fast - s0.docs_fast,
                          "docs_per_s": round(n / ms * 1e3), "algo_GBps": round(algo / ms / 1e6, 1), "gen_s": round(gen, 1)}))


def c2del(n):
    arena, upd_off, doc_upd = synth.text_updates(n, 200, seed=5, del_pct=20)
    e = Engine(0)
    da = dev(np.concatenate([arena, np.zeros(64, np.uint8)]))
    do = dev(upd_off.view(np.int64))
    dd = dev(doc_upd.view(np.int32))
    for rep in range(4):
        s0 = e.stats()
        r = e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), n)
        s1 = e.stats()
    ms = s1.kernel_ms - s0.kernel_ms
    algo = len(arena) + r.payload_bytes
    print(json.dumps({"config": "C2+20%del", "op": "merge", "docs": n, "kernel_ms": round(ms, 3), "docs_per_s": round(n / ms * 1e3),
                      "algo_GBps": round(algo / ms / 1e6, 1), "lean_docs": s1.docs_lean - s0.docs_lean, "seq_docs": s1.docs_seq - s0.docs_seq}))


def big(n, max_bytes, xml):
    t0 = time.time()
    if xml:
        arena, upd_off, doc_upd = synth.big_docs(n, max_bytes, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
    else:
        arena, upd_off, doc_upd = synth.big_docs(n, max_bytes, 1024, max_clients=64, max_k=200, seed=8)
    gen = time.time() - t0
    e = Engine(0)
    da = dev(np.concatenate([arena, np.zeros(64, np.uint8)]))
    do = dev(upd_off.view(np.int64))
    dd = dev(doc_upd.view(np.int32))
    sizes = np.diff(upd_off[doc_upd].astype(np.int64))
    for rep in range(2):
        s0 = e.stats()
        t = time.time()
        r = e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), n)
        wall = time.time() - t
        s1 = e.stats()
    ms = s1.kernel_ms - s0.kernel_ms
    algo = len(arena) + r.payload_bytes
    print(json.dumps({"config": "C5" if xml else "C3", "op": "merge", "docs": n, "bytes_in": len(arena),
                      "largest_doc": int(sizes.max()), "kernel_ms": round(ms, 3), "wall_ms": round(wall * 1e3, 3),
                      "docs_per_s": round(n / ms * 1e3), "algo_GBps": round(algo / ms / 1e6, 2),
                      "lean_docs": s1.docs_lean - s0.docs_lean, "fast_docs": s1.docs_fast - s0.docs_fast,
                      "seq_docs": s1.docs_seq - s0.docs_seq, "gen_s": round(gen, 1)}))


if __name__ == "__main__":
    which = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    if which in ("c3", "c5"):
        big(n, int(float(sys.argv[3])) if len(sys.argv) > 3 else 1_000_000, which == "c5")
    else:
        {"c4": c4, "c2del": c2del}[which](n)
