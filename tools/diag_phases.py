"""Phase breakdown of the merge kernels on the C2 workload (diagnostic build libygm_diag.so; tooling, not product).

k_merge_lean: absolute shader-clock stamps per document (no atomics) -> mean phase durations,
kernel span and mean number of documents in flight.  k_merge_wave / k_merge_fast: atomic sums."""
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
mixed = len(sys.argv) > 2 and sys.argv[2] == "mixed"   # the c2_mixed corpus: stamps of the wide kernel's waves
if mixed:
    arena, upd_off, doc_upd = synth.text_updates(n_docs, 200, 1, 8, del_pct=20, seed=71, max_run=16)
else:
    arena, upd_off, doc_upd = synth.text_updates(n_docs, 200, seed=1000)
upd_doc = np.repeat(np.arange(n_docs, dtype=np.uint32), np.diff(doc_upd).astype(np.int64))
e = eng.Engine(0)
L = eng.lib()
L.ygm_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.ygm_diag_ts_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(64, np.uint64)
ts = np.zeros(16384 * 8, np.uint64)
for rep in range(3):
    L.ygm_diag_read(buf.ctypes.data, 1)
    e.merge_packed(arena, upd_off, upd_doc, n_docs)
    L.ygm_diag_read(buf.ctypes.data, 0)
L.ygm_diag_ts_read(ts.ctypes.data, 0)
t = ts.reshape(16384, 8)[:min(n_docs, 1500 if mixed else 16384)].astype(np.int64)
# slots: 0 start, 6 header loaded, 1 staged, 2 parsed, 3 scanned, 4 emitted, 8 end (s_memrealtime, 100 MHz -> ns x10)
print("k_merge_lean - ns per document (mean; s_memrealtime stamps):")
order = [("stage", 1), ("parse", 2), ("clients+scan", 3), ("emit", 4), ("tail", 8)]
prev = t[:, 0]
for nm, c in order:
    col = t[:, c] if c < 8 else None
    if col is None:
        break
    ok = col > 0
    print(f"  {nm:26s} {10.0 * np.mean(col[ok] - prev[ok]):10.0f}")
    prev = np.where(ok, col, prev)
ds = t[:, 7] - t[:, 6]
okd = (t[:, 6] > 0) & (t[:, 7] >= t[:, 6])
print(f"  of which: parsed -> delete-set union {10.0 * np.mean((t[:, 6] - t[:, 2])[okd]):.0f}, the union {10.0 * np.mean(ds[okd]):.0f}, "
      f"union -> scanned {10.0 * np.mean((t[:, 3] - t[:, 7])[okd]):.0f}")
life = np.max(t[:, 1:6], axis=1) - t[:, 0]
span = np.max(t[:, 1:6]) - np.min(t[:, 0])
print(f"  lifetime mean {10.0 * life.mean():.0f} ns  kernel span {10.0 * span:.0f} ns  mean docs in flight {life.sum() / max(span, 1):.1f}")
st = np.sort(t[:, 0] - t[:, 0].min())
print("  start-time percentiles (ns) 10/50/90/100:", [int(10 * np.percentile(st, p)) for p in (10, 50, 90, 100)])
for title, nms, lo in (("k_merge_wave (wave per document)", ["stage", "parse", "clients+sort", "classify+scan", "-", "deleteset", "-", "emit"], 8),
                       ("k_merge_fast (workgroup per document)", ["stage", "passA", "scan+passB", "sort", "classify", "deleteset", "place", "emit"], 0)):
    tot = buf[lo:lo + 8].sum()
    if tot == 0:
        continue
    print(title, "- shader cycles per document (mean, last rep):")
    for i, nm in enumerate(nms):
        print(f"  {nm:16s} {buf[lo + i] / n_docs:12.0f}  {100.0 * buf[lo + i] / max(tot, 1):5.1f}%")
if mixed:
    L.ygm_diag_ds_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dsb = np.zeros(4, np.uint64)
    L.ygm_diag_ds_read(dsb.ctypes.data, 0)
    print("delete-set union, shader cycles per document (3 reps): records", int(dsb[0]) // (3 * n_docs), "rank sort",
          int(dsb[1]) // (3 * n_docs), "runs/scans", int(dsb[2]) // (3 * n_docs))
s = e.stats()
print("kernel_ms (3 reps)", s.kernel_ms, "lean_ms", s.lean_ms, "docs_lean", s.docs_lean)
