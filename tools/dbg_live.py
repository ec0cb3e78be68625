"""Debug probe (tooling): live-session documents (tools/synth_live.c) merged on the GPU one at a time, each compared
with the oracle; prints the tier that took the document (stats deltas), the first differing byte and context.

    python tools/dbg_live.py [c5|c3] n_docs max_bytes [seed] [135]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import oracle
    from hocuspocus_amd import Engine
    from tools import synth
    kind = sys.argv[1]
    n, mb = int(sys.argv[2]), float(sys.argv[3])
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else (5 if kind == "c5" else 3)
    c135 = len(sys.argv) > 5 and sys.argv[5] == "135"
    if kind == "c5":
        a, uo, du = synth.live_docs(n, int(mb), min_bytes=64 * 1024, n_clients=10000, xml=True, max_k=50, seed=seed)
    else:
        a, uo, du = synth.live_docs(n, int(mb), min_bytes=1 << 20, n_clients=64, max_k=200, seed=seed)
    ups = synth.split(a, uo)
    docs = [ups[du[d]:du[d + 1]] for d in range(n)]
    for force_seq in (False, True):
        e = Engine(0, compat135=c135, force_seq=force_seq)
        for d, us in enumerate(docs):
            s0 = e.stats()
            got = e.merge_updates_batch([us])[0]
            s1 = e.stats()
            exp = oracle.merge_updates(us, compat135=c135)
            rec = {"doc": d, "force_seq": force_seq, "updates": len(us), "in_bytes": sum(map(len, us)), "ok": got == exp,
                   "tiers": {k: getattr(s1, k) - getattr(s0, k) for k in ("docs_lean", "docs_fast", "docs_big", "docs_seq")},
                   "status": [got[0], exp[0]]}
            if got != exp and got[1] is not None and exp[1] is not None:
                g, x = got[1], exp[1]
                i = next((i for i in range(min(len(g), len(x))) if g[i] != x[i]), min(len(g), len(x)))
                rec.update(len=[len(g), len(x)], first_diff=i, got=g[max(0, i - 24):i + 24].hex(), exp=x[max(0, i - 24):i + 24].hex())
            print(json.dumps(rec), flush=True)
        e.close()


if __name__ == "__main__":
    main()
