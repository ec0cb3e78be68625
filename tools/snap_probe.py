"""Snapshot-kernel probe (tooling): the time of ygm_snapshot_v1_device on live-session documents (tools/synth_live.c)
by size and shape -- the general snapshot kernel runs one thread per document, so a batch takes about its largest
document's time.  One JSON line per (shape, size): kernel ms for a batch of `n` documents of that size.

    python tools/snap_probe.py [n]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import oracle
    from hocuspocus_amd import Engine
    from tools import synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    e = Engine(0)
    shapes = (("xml_10k_clients", dict(n_clients=10000, xml=True)), ("xml_300_clients", dict(n_clients=300, xml=True)),
              ("text_64_clients", dict(n_clients=64)), ("text_4_clients", dict(n_clients=4)))
    for name, kw in shapes:
        for kb in (4, 16, 64, 256, 1024):
            if kw.get("n_clients", 0) >= 10000 and kb < 512:
                continue   # (10 000 client blocks need ~400 KB)
            a, uo, du = synth.live_docs(n, kb * 1024, min_bytes=kb * 1024, max_k=20, seed=kb, **kw)
            ups = synth.split(a, uo)
            states = [oracle.merge_updates(ups[du[d]:du[d + 1]])[1] for d in range(n)]
            arena = np.frombuffer(b"".join(states) + bytes(64), np.uint8)
            off = np.cumsum([0] + [len(s) for s in states]).astype(np.uint64)
            da = torch.from_numpy(arena.copy()).to(dev)
            do = torch.from_numpy(off.view(np.int64)).to(dev)
            best = None
            for _ in range(2):
                s0 = e.stats()
                r = e.snapshot_device(da.data_ptr(), len(arena) - 64, do.data_ptr(), n)
                torch.cuda.synchronize()
                ms = e.stats().kernel_ms - s0.kernel_ms
                best = ms if best is None or ms < best else best
            print(json.dumps({"shape": name, "kb": kb, "docs": n, "bytes": int(off[-1]), "snapshot_ms": round(best, 2),
                              "us_per_byte_of_largest": round(best * 1e3 / max(len(s) for s in states), 3)}), flush=True)
            if best > 15000:
                break


if __name__ == "__main__":
    main()
