"""C3 / C5 tier probe (diagnostic build libygm_diag.so; tooling): documents per tier and the
k_merge_fast / k_merge_wave phase sums (shader cycles) on the bench's C3 or C5 corpus."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hocuspocus_amd.engine as eng  # noqa: E402

eng.LIB_PATH = os.path.join(ROOT, "hocuspocus_amd", "libygm_diag.so")
from tools import synth  # noqa: E402

xml = len(sys.argv) > 1 and sys.argv[1] == "c5"
if xml:
    arena, upd_off, doc_upd = synth.big_docs(20, 1_000_000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
else:
    arena, upd_off, doc_upd = synth.big_docs(2000, 1_000_000, 1024, max_clients=64, max_k=200, seed=8)
n = len(doc_upd) - 1
sizes = np.diff(upd_off[doc_upd].astype(np.int64))
ks = np.diff(doc_upd.astype(np.int64))
print("docs", n, "bytes", len(arena), "size pct 50/90/99/max", [int(np.percentile(sizes, p)) for p in (50, 90, 99, 100)],
      "k pct 50/90/max", [int(np.percentile(ks, p)) for p in (50, 90, 100)])
print("docs > 16 KB", int((sizes > 16384).sum()), "docs > 64 KB", int((sizes > 65536).sum()))
upd_doc = np.repeat(np.arange(n, dtype=np.uint32), ks)
e = eng.Engine(0)
L = eng.lib()
L.ygm_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(64, np.uint64)
e.merge_packed(arena, upd_off, upd_doc, n)
L.ygm_diag_read(buf.ctypes.data, 1)
s0 = e.stats()
e.merge_packed(arena, upd_off, upd_doc, n)
s1 = e.stats()
L.ygm_diag_read(buf.ctypes.data, 0)
print("kernel_ms", round(s1.kernel_ms - s0.kernel_ms, 3), "lean_ms", round(s1.lean_ms - s0.lean_ms, 3),
      "docs lean", s1.docs_lean - s0.docs_lean, "fast", s1.docs_fast - s0.docs_fast, "big", s1.docs_big - s0.docs_big,
      "seq", s1.docs_seq - s0.docs_seq)
for title, nms, lo in (("k_merge_wave", ["stage", "parse", "clients+sort", "classify+scan", "-", "deleteset", "-", "emit"], 8),
                       ("k_merge_fast", ["stage", "passA", "scan+passB", "sort", "classify", "deleteset", "place", "emit"], 0)):
    tot = buf[lo:lo + 8].sum()
    print(title, "total Mcycles", round(tot / 1e6, 2), {nm: round(buf[lo + i] / 1e6, 2) for i, nm in enumerate(nms)})
