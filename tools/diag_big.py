"""Phase breakdown of k_merge_big on C5 documents (diagnostic build libygm_diag.so; tooling).
Stamps (s_memrealtime, 100 MHz) per document: start, log walk, U0 walk, sorts, pass 0, pass 1."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hocuspocus_amd.engine as eng  # noqa: E402

eng.LIB_PATH = os.path.join(ROOT, "hocuspocus_amd", "libygm_diag.so")
from tools import synth  # noqa: E402

xml = len(sys.argv) > 1 and sys.argv[1] in ("c5", "c5full")
if len(sys.argv) > 1 and sys.argv[1] == "c5full":   # the bench's C5 block (1 000 documents: four mid workgroups per CU)
    arena, upd_off, doc_upd = synth.big_docs(1000, 1_000_000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
elif len(sys.argv) > 1 and sys.argv[1] == "c3dev":   # the bench's C3 full block, through the device API (one launch per size)
    arena, upd_off, doc_upd = synth.big_docs(100000, 10_000_000, 1024, max_clients=64, max_k=200, seed=8)
elif len(sys.argv) > 1 and sys.argv[1] == "c3top":   # the C3 corpus' largest documents (10 MB * rank^-0.8: the 16-wave size)
    arena, upd_off, doc_upd = synth.big_docs(8, 10_000_000, 1024, max_clients=64, max_k=200, seed=8)
elif xml:
    arena, upd_off, doc_upd = synth.big_docs(20, 600000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
else:
    arena, upd_off, doc_upd = synth.big_docs(200, 300000, 1024, max_clients=64, max_k=200, seed=8)
n = len(doc_upd) - 1
upd_doc = np.repeat(np.arange(n, dtype=np.uint32), np.diff(doc_upd).astype(np.int64))
e = eng.Engine(0)
L = eng.lib()
L.ygm_diag_ts_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
ts = np.zeros(16384 * 8, np.uint64)
if len(sys.argv) > 1 and sys.argv[1] in ("c3dev", "c5full"):
    import torch
    dev = torch.device("cuda", 0)
    da = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).to(dev)
    do = torch.from_numpy(upd_off.view(np.int64)).to(dev)
    dd = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
    for _ in range(2):
        e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), n)
    torch.cuda.synchronize()
else:
    e.merge_packed(arena, upd_off, upd_doc, n)
    e.merge_packed(arena, upd_off, upd_doc, n)
L.ygm_diag_ts_read(ts.ctypes.data, 0)
L.ygm_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
cnt = np.zeros(32, np.uint64)
L.ygm_diag_read(cnt.ctypes.data, 0)
# follow counts over both runs (slots 16-20): client blocks, jump steps, structs taken by them, structs parsed
# from global memory, block headers that took the cursor parse
print("follow counts (2 runs): blocks", int(cnt[16]), "jump steps", int(cnt[17]), "structs by jump", int(cnt[18]),
      "global parses", int(cnt[19]), "slow headers", int(cnt[20]))
st = e.stats()
print("docs_big", st.docs_big, "docs_seq", st.docs_seq)
# follow time by part over both runs (slots 25-28, wave 0 shader cycles): tile loads + spec, block headers, struct
# steps, block tails
print("follow cycles (2 runs): tile", int(cnt[25]), "headers", int(cnt[26]), "structs", int(cnt[27]), "tails", int(cnt[28]),
      "per block:", {k: round(int(cnt[i]) / max(int(cnt[16]), 1), 1) for k, i in (("tile", 25), ("hdr", 26), ("st", 27), ("tail", 28))})
# the speculative parse by part (slots 29-31, lane 0 of wave 0, 100 MHz ticks): nx fill + first jump level, the
# other levels, the block table
print("spec ticks (2 runs): nx+jp0", int(cnt[29]), "jp1..", int(cnt[30]), "block table", int(cnt[31]))
t = ts.reshape(16384, 8)[:n].astype(np.int64)
# stamps: start, log walk, U0 walk, sorts, pass0, pass1; slots 6 / 7: time inside the U0 walk spent in
# the speculative tile parse / in validation
d = np.diff(t[:, :6], axis=1) * 10 / 1000.0   # us
d = np.concatenate([d[:, :1], d[:, 1:2] - (t[:, 6:8].sum(1, keepdims=True) * 10 / 1000.0), t[:, 6:8] * 10 / 1000.0, d[:, 2:]], axis=1)
names = ["log walk", "U0 follow", "U0 spec parse", "U0 validate", "sorts", "pass0", "pass1"]
sizes = np.diff(upd_off[doc_upd].astype(np.int64))
tot = d.sum(1)
live = t[:, 0] > 0
print("per-document total us percentiles 10/50/90/99 (rows written):", np.round(np.percentile(tot[live], [10, 50, 90, 99]), 1).tolist(),
      "phase medians:", dict(zip(names, np.round(np.median(d[live], 0), 1))))
for q in np.argsort(-d.sum(1))[:5]:
    print("block", q, "us", dict(zip(names, np.round(d[q], 1))))
print("mean us", dict(zip(names, np.round(d.mean(0), 1))), "max total us", round(d.sum(1).max(), 1), "bytes max", sizes.max())
# concurrency: start / end stamps of the workgroups (row = blockIdx; the last kernel to write a row wins)
ok = t[:, 0] > 0
if ok.any():
    st, en = t[ok, 0], t[ok, 5]
    z = st.min()
    print("start us percentiles 0/25/50/75/100:", np.round(np.percentile((st - z) * 10 / 1000.0, [0, 25, 50, 75, 100]), 1).tolist(),
          "end:", np.round(np.percentile((en - z) * 10 / 1000.0, [0, 25, 50, 75, 100]), 1).tolist(),
          "per-doc total us median:", round(float(np.median(d[ok].sum(1))), 1))
    rows = np.nonzero(ok)[0]
    sb = ((st - z) * 10 / 1000.0 // 1000).astype(int)
    eb = ((en - z) * 10 / 1000.0 // 1000).astype(int)
    print("start histogram (ms bin: count):", dict(zip(*np.unique(sb, return_counts=True))))
    print("end histogram (ms bin: count):", dict(zip(*np.unique(eb, return_counts=True))))
    late = rows[sb >= 5]
    print("late rows (blockIdx) first/last/count:", late[:8].tolist(), late[-8:].tolist(), len(late))
