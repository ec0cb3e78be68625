"""Merge-kernel variant probe (tooling): device merge timings of one or more experiment builds of
libygm.so on C2-shaped corpora, each output digested (sha256 over status + bytes of every document in
order) so a variant can be compared with the product build the parity tests pin.

    python tools/exp_lean.py lib1.so [lib2.so ...]

Corpora: C2 100k docs (1-4 clients), C2 10k, C2 100k with 20 % deletions, C2 100k with 5-8 clients.
Each library runs in its own child process (one libygm per process); one JSON line per (lib, corpus)."""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORPORA = [("c2_100k", 100000, dict()), ("c2_10k", 10000, dict()), ("c2_del20_100k", 100000, dict(del_pct=20)),
           ("c2_8cl_100k", 100000, dict(min_clients=5, max_clients=8))]


def child(which):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from bench import _d2h
    from hocuspocus_amd import Engine
    from tools import synth
    dev = torch.device("cuda", 0)
    e = Engine(0)
    for name, n, kw in CORPORA:
        if which and name not in which:
            continue
        arena, upd_off, doc_upd = synth.text_updates(n, 200, seed=1000, **kw)
        da = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).to(dev)
        do = torch.from_numpy(upd_off.view(np.int64)).to(dev)
        dd = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
        best = None
        for rep in range(8):
            s0 = e.stats()
            r = e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), n)
            s1 = e.stats()
            ms = s1.lean_ms - s0.lean_ms
            best = ms if best is None or ms < best else best
        torch.cuda.synchronize()
        st = _d2h(r.status, n * 4).view(np.int32)
        off = _d2h(r.off, n * 8).view(np.uint64)
        ln = _d2h(r.len, n * 8).view(np.uint64)
        data = _d2h(r.data, int(off.max() + ln.max()) + 16)
        h = hashlib.sha256(st.tobytes())
        for d in range(n):
            p = data[int(off[d]):int(off[d]) + int(ln[d])].tobytes() if st[d] == 0 else b""
            h.update(len(p).to_bytes(4, "little"))
            h.update(p)
        algo = len(arena) + int(r.payload_bytes)
        print(json.dumps({"lib": os.path.basename(os.environ.get("YGM_LIB", "libygm.so")), "corpus": name, "docs": n,
                          "lean_best_ms": round(best, 4), "total_ms": round(s1.kernel_ms - s0.kernel_ms, 4),
                          "algo_GBps": round(algo / best / 1e6, 1), "frac": round(algo / best / 1e6 / 8000, 4),
                          "lean_docs": s1.docs_lean - s0.docs_lean, "digest": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] else None)
        sys.exit(0)
    which = os.environ.get("EXP_CORPORA", "")
    for lib in sys.argv[1:]:
        env = dict(os.environ, YGM_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", which], env=env, timeout=400)
        if r.returncode != 0:
            print(json.dumps({"lib": lib, "error": r.returncode}), flush=True)
            sys.exit(r.returncode)
