"""Kernel-variant probe (tooling): C4 state vector + diff timings of one or more experiment builds of
libygm.so on the same corpus, each output digested (sha256 over status + bytes of every document in
order) so a variant can be compared with the product build that the parity tests pin.

    python tools/exp_c4.py n_docs lib1.so[@VAR=v,VAR=v] [lib2.so ...]

Each library runs in its own child process (one libygm per process, with the environment variables named after
@); prints one JSON line per (lib, op).  Per-document output hashes are kept: documents whose output differs from
the first library's are counted and up to 4 of them checked against the CPU oracle."""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(n):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from bench import _d2h
    from hocuspocus_amd import Engine
    from tools import synth
    arena, doc_off, sva, sv_off = synth.text_states(n, seed=3)
    dev = torch.device("cuda", 0)

    def put(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    da = put(np.concatenate([arena, np.zeros(64, np.uint8)]))
    do = put(doc_off.view(np.int64))
    ds = put(np.concatenate([sva, np.zeros(64, np.uint8)]))
    dso = put(sv_off.view(np.int64))
    e = Engine(0)
    for op in ("sv", "diff"):
        best = None
        for rep in range(5):
            s0 = e.stats()
            r = e.sv_device(da, len(arena), do, n) if op == "sv" else e.diff_device(da, len(arena), do, ds, dso, n)
            s1 = e.stats()
            ms = s1.kernel_ms - s0.kernel_ms
            best = ms if best is None or ms < best else best
        torch.cuda.synchronize()
        st = _d2h(r.status, n * 4).view(np.int32)
        off = _d2h(r.off, n * 8).view(np.uint64)
        ln = _d2h(r.len, n * 8).view(np.uint64)
        data = _d2h(r.data, int(r.data_bytes))
        h = hashlib.sha256(st.tobytes())
        # document outputs in document order (offsets are slot-relative and may differ between variants)
        order = np.argsort(off, kind="stable")
        pieces = [None] * n
        for d in order:
            pieces[d] = data[int(off[d]):int(off[d]) + int(ln[d])].tobytes() if st[d] == 0 else b""
        dh = np.zeros(n, np.uint64)
        for d, p in enumerate(pieces):
            h.update(len(p).to_bytes(4, "little"))
            h.update(p)
            dh[d] = int.from_bytes(hashlib.blake2b(p + bytes([st[d] & 255]), digest_size=8).digest(), "little")
        np.save(os.path.join(os.environ["EXP_C4_DUMP"], f"{op}.npy"), dh)
        algo = len(arena) + int(r.payload_bytes) + (len(sva) if op == "diff" else 0)
        print(json.dumps({"lib": os.path.basename(os.environ.get("YGM_LIB", "libygm.so")), "op": op, "docs": n,
                          "best_ms": round(best, 3), "last_ms": round(ms, 3), "algo_GBps": round(algo / best / 1e6, 1),
                          "walker_docs": s1.docs_lean - s0.docs_lean, "digest": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]))
        sys.exit(0)
    import tempfile

    import numpy as np
    n = int(sys.argv[1])
    dumps = []
    for spec in sys.argv[2:]:
        lib, _, envs = spec.partition("@")
        env = dict(os.environ, YGM_LIB=os.path.abspath(lib))
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        dump = tempfile.mkdtemp(prefix="exp_c4_")
        env["EXP_C4_DUMP"] = dump
        dumps.append((spec, dump))
        print(json.dumps({"spec": spec}), flush=True)
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", str(n)], env=env, timeout=240)
        if r.returncode != 0:
            print(json.dumps({"lib": lib, "error": r.returncode}), flush=True)
            sys.exit(r.returncode)
    if len(dumps) > 1:
        sys.path.insert(0, ROOT)
        import oracle
        from tools import synth
        arena, doc_off, sva, sv_off = synth.text_states(n, seed=3)
        for op in ("sv", "diff"):
            base = np.load(os.path.join(dumps[0][1], f"{op}.npy"))
            for spec, dump in dumps[1:]:
                x = np.load(os.path.join(dump, f"{op}.npy"))
                bad = np.nonzero(x != base)[0]
                rec = {"op": op, "spec": spec, "differs_from_first": int(len(bad)), "first_docs": bad[:4].tolist()}
                if len(bad):   # which one the oracle agrees with (the bytes are re-derived: hashes only were kept)
                    rec["oracle_check"] = []
                    for d in bad[:4].tolist():
                        u = bytes(arena[doc_off[d]:doc_off[d + 1]])
                        ex = oracle.encode_state_vector_from_update(u) if op == "sv" else oracle.diff_update(u, bytes(sva[sv_off[d]:sv_off[d + 1]]))
                        eh = int.from_bytes(hashlib.blake2b((ex[1] if ex[0] == 0 else b"") + bytes([ex[0] & 255]), digest_size=8).digest(), "little")
                        rec["oracle_check"].append({"doc": d, "first_ok": bool(eh == base[d]), "this_ok": bool(eh == x[d])})
                print(json.dumps(rec), flush=True)
