"""Phase breakdown of the merge kernels on the C2 workload (diagnostic build libygm_diag.so; tooling, not product)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hocuspocus_amd.engine as eng  # noqa: E402

eng.LIB_PATH = os.path.join(ROOT, "hocuspocus_amd", "libygm_diag.so")
from tools import synth  # noqa: E402

n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
arena, upd_off, doc_upd = synth.text_updates(n_docs, 200, seed=1000)
upd_doc = np.repeat(np.arange(n_docs, dtype=np.uint32), np.diff(doc_upd).astype(np.int64))
e = eng.Engine(0)
L = eng.lib()
L.ygm_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(16, np.uint64)
for rep in range(3):
    L.ygm_diag_read(buf.ctypes.data, 1)
    e.merge_packed(arena, upd_off, upd_doc, n_docs)
    L.ygm_diag_read(buf.ctypes.data, 0)
for title, names, lo in (("k_merge_wave (wave per document)", ["stage", "parse", "clients+sort", "classify+scan", "-", "deleteset", "-", "emit"], 8),
                         ("k_merge_fast (workgroup per document)", ["stage", "passA", "scan+passB", "sort", "classify", "deleteset", "place", "emit"], 0)):
    tot = buf[lo:lo + 8].sum()
    if tot == 0:
        continue
    print(title, "- shader cycles per document (mean, last rep):")
    for i, nm in enumerate(names):
        print(f"  {nm:16s} {buf[lo + i] / n_docs:12.0f}  {100.0 * buf[lo + i] / max(tot, 1):5.1f}%")
s = e.stats()
print("kernel_ms (3 reps)", s.kernel_ms)
