"""Walker probe for profiler passes (tooling): C4 state vector / diff launches of the library named by YGM_LIB
(default hocuspocus_amd/libygm.so) on the 1M-document corpus, no output hashing, so a rocprofv3 --pmc pass over it
is short.

    python tools/walk_probe.py n_docs [sv|diff|both] [reps]

Prints one JSON line per op with the best kernel time (HIP events inside the engine)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from hocuspocus_amd import Engine
    from tools import synth
    n = int(sys.argv[1])
    ops = ("sv", "diff") if len(sys.argv) < 3 or sys.argv[2] == "both" else (sys.argv[2],)
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    arena, doc_off, sva, sv_off = synth.text_states(n, seed=3)
    dev = torch.device("cuda", 0)

    def put(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    da = put(np.concatenate([arena, np.zeros(64, np.uint8)]))
    do = put(doc_off.view(np.int64))
    ds = put(np.concatenate([sva, np.zeros(64, np.uint8)]))
    dso = put(sv_off.view(np.int64))
    e = Engine(0)
    for op in ops:
        best = None
        for _ in range(reps):
            s0 = e.stats()
            r = e.sv_device(da, len(arena), do, n) if op == "sv" else e.diff_device(da, len(arena), do, ds, dso, n)
            s1 = e.stats()
            ms = s1.kernel_ms - s0.kernel_ms
            best = ms if best is None or ms < best else best
        torch.cuda.synchronize()
        print(json.dumps({"lib": os.path.basename(os.environ.get("YGM_LIB", "libygm.so")), "op": op, "docs": n,
                          "best_ms": round(best, 3), "payload": int(r.payload_bytes),
                          "walker_docs": s1.docs_lean - s0.docs_lean}), flush=True)


if __name__ == "__main__":
    main()
