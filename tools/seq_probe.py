"""Sequential-tier probe (tooling): one large [snapshot, ...log] document forced through the exact
sequential kernel with short and long logs; wall ms per merge."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hocuspocus_amd import Engine  # noqa: E402
from tools import synth  # noqa: E402

arena, upd_off, doc_upd = synth.big_docs(1, 300000, 1024, max_clients=8, max_k=200, seed=31)
ups = synth.split(arena, upd_off)
snap, log = ups[0], ups[1:]
e = Engine(0, force_seq=True)
for k in (1, 2, 10, 50, len(log)):
    batch = [[snap] + log[:k]]
    e.merge_updates_batch(batch)
    t = time.time()
    r = e.merge_updates_batch(batch)
    print("k", k + 1, "bytes", len(snap), "status", r[0][0], "ms", round((time.time() - t) * 1e3, 2), flush=True)
