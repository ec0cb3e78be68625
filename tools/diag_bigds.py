"""k_merge_big emit split (diagnostic build with -DYGM_DIAG -DYGM_DIAG_BIGDS; tooling): per document, pass 0 / pass 1
time in the block merge vs the delete-set merge, on the bench's C3 or C5 corpus (largest documents first)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hocuspocus_amd.engine as eng  # noqa: E402

eng.LIB_PATH = os.path.abspath(sys.argv[2]) if len(sys.argv) > 2 else os.path.join(ROOT, "hocuspocus_amd", "libygm_diag.so")
from tools import synth  # noqa: E402

xml = sys.argv[1] == "c5"
if xml:
    arena, upd_off, doc_upd = synth.big_docs(20, 1_000_000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
else:
    arena, upd_off, doc_upd = synth.big_docs(2000, 1_000_000, 1024, max_clients=64, max_k=200, seed=8)
n = len(doc_upd) - 1
upd_doc = np.repeat(np.arange(n, dtype=np.uint32), np.diff(doc_upd).astype(np.int64))
e = eng.Engine(0)
L = eng.lib()
L.ygm_diag_ts_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
ts = np.zeros(16384 * 8, np.uint64)
e.merge_packed(arena, upd_off, upd_doc, n)
e.merge_packed(arena, upd_off, upd_doc, n)
L.ygm_diag_ts_read(ts.ctypes.data, 0)
st = e.stats()
t = ts.reshape(16384, 8)[:st.docs_big // 2 if st.docs_big else n].astype(np.int64)
us = lambda x: np.round(x * 10 / 1000.0, 1)   # noqa: E731  (s_memrealtime: 100 MHz)
tot = t[:, 5] - t[:, 0]
for q in np.argsort(-tot)[:6]:
    r = t[q]
    print(f"wg {q}: total {us(r[5] - r[0])} us | log {us(r[1] - r[0])} U0 walk {us(r[2] - r[1])} sorts {us(r[3] - r[2])} | "
          f"pass0 blocks {us(r[6] - r[3])} ds {us(r[4] - r[6])} | pass1 blocks {us(r[7] - r[4])} ds {us(r[5] - r[7])}")
# medians over every large-tier workgroup row written, and the delete-set plan counters (slots 21 / 22: documents
# planned, documents on the spliced path)
ok = t[:, 0] > 0
if ok.any():
    r = t[ok]
    parts = {"log": r[:, 1] - r[:, 0], "U0 walk": r[:, 2] - r[:, 1], "sorts": r[:, 3] - r[:, 2], "pass0 blocks": r[:, 6] - r[:, 3],
             "pass0 ds": r[:, 4] - r[:, 6], "pass1 blocks": r[:, 7] - r[:, 4], "pass1 ds": r[:, 5] - r[:, 7]}
    print("rows", int(ok.sum()), "median us", {k: float(us(np.median(v))) for k, v in parts.items()},
          "mean us", {k: float(us(np.mean(v))) for k, v in parts.items()})
L.ygm_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
cnt = np.zeros(32, np.uint64)
L.ygm_diag_read(cnt.ctypes.data, 0)
print("ds plan: documents", int(cnt[21]), "spliced", int(cnt[22]))
