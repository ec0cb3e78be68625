"""Throughput probes for the non-headline configs (tooling; bench.py stays the C2 contract).

    python tools/bench_configs.py c4 [n_docs]     state vector + diffUpdate over synthetic merged states (C4)
    python tools/bench_configs.py c2del [n_docs]  C2 with 20 % deletes (deferred tiers)
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


if __name__ == "__main__":
    which = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    {"c4": c4, "c2del": c2del}[which](n)
