"""Dev probe (tooling): k_merge_big on single large C3-shaped documents (device API, kernel ms) and the diag build's
per-phase stamps of the same documents.   python tools/proto/big_probe.py [diag]"""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
diag = len(sys.argv) > 1 and sys.argv[1] in ("diag", "diagds", "splice", "occ")
dsmode = len(sys.argv) > 1 and (sys.argv[1] == "diagds" or (sys.argv[1] == "occ" and os.environ.get("OCC_DS") == "1"))
import hocuspocus_amd.engine as eng
if diag:
    eng.LIB_PATH = os.path.join(ROOT, "hocuspocus_amd", "exp/libygm_diagds.so" if dsmode else "libygm_diag.so")
from tools import synth
import oracle
e = eng.Engine(0)
if len(sys.argv) > 1 and sys.argv[1] == "tiers":   # the full C3 batch: documents and time per tier
    arena, upd_off, doc_upd = synth.big_docs(100000, 10_000_000, 1024, max_clients=64, max_k=200, seed=8)
    n = 100000
    upd_doc = np.repeat(np.arange(n, dtype=np.uint32), np.diff(doc_upd).astype(np.int64))
    for rep in range(3):
        s0 = e.stats(); t0 = time.time()
        e.merge_packed_raw(arena, upd_off, upd_doc, n)
        s1 = e.stats()
    print({k: round(getattr(s1, k) - getattr(s0, k), 3) for k in ("kernel_ms", "lean_ms", "docs_lean", "docs_lean_wide", "docs_fast", "docs_big", "docs_seq")}, flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "occ":   # C3-full-shaped batch (top ranks): per-workgroup stamps -> concurrency
    n = int(os.environ.get("OCC_N", "16000"))
    arena, upd_off, doc_upd = synth.big_docs(n, 10_000_000, 1024, max_clients=64, max_k=200, seed=8)
    upd_doc = np.repeat(np.arange(n, dtype=np.uint32), np.diff(doc_upd).astype(np.int64))
    L = eng.lib()
    L.ygm_diag_ts_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for rep in range(2):
        s0 = e.stats()
        res = e.merge_packed_raw(arena, upd_off, upd_doc, n)
        s1 = e.stats()
    ts = np.zeros(16384 * 8, np.uint64)
    L.ygm_diag_ts_read(ts.ctypes.data, 0)
    nb = s1.docs_big - s0.docs_big
    t = ts.reshape(16384, 8).astype(np.int64)[: min(nb, 16384)]
    t = t[t[:, 0] > 0]
    st, en = t[:, 0], t[:, 5]
    ok = en > st
    st, en, tt = st[ok], en[ok], t[ok]
    span = (en.max() - st.min()) / 100.0   # us
    busy = (en - st).sum() / 100.0
    ph = np.diff(tt[:, :6], axis=1).sum(axis=0) / 100.0
    if dsmode:   # slots 6 / 7: the delete-set part's start in each pass
        ds = {"pass0 structs": (tt[:, 6] - tt[:, 3]).sum() / 100.0, "pass0 ds": (tt[:, 4] - tt[:, 6]).sum() / 100.0,
              "pass1 structs": (tt[:, 7] - tt[:, 4]).sum() / 100.0, "pass1 ds": (tt[:, 5] - tt[:, 7]).sum() / 100.0}
        print({"ds_split_us": ds}, flush=True)
    sizes = np.diff(upd_off[doc_upd].astype(np.int64))
    print({"docs": n, "bytes": int(upd_off[-1]), "kernel_ms": round(s1.kernel_ms - s0.kernel_ms, 2), "docs_big": int(nb),
           "wg_stamped": int(ok.sum()), "span_us": round(span, 1), "busy_wg_us": round(busy, 1), "mean_concurrency": round(busy / span, 1),
           "phase_sum_us": {"log": ph[0], "u0": ph[1], "sorts": ph[2], "pass0": ph[3], "pass1": ph[4]},
           "median_doc_bytes": int(np.median(sizes)), "wg_us_p50_p99_max": [float(np.percentile((en - st) / 100.0, q)) for q in (50, 99, 100)]}, flush=True)
    # concurrency timeline: 20 buckets
    t0 = st.min(); edges = np.linspace(0, en.max() - t0, 21)
    conc = [int(((st - t0 <= (a + b) / 2) & (en - t0 >= (a + b) / 2)).sum()) for a, b in zip(edges[:-1], edges[1:])]
    print({"concurrency_timeline": conc}, flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "splice":   # tests/tile_docs.ds_splice_docs through the diag build
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from tile_docs import ds_splice_docs
    L = eng.lib()
    L.ygm_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dg = np.zeros(32, np.uint64)
    for seed in (11, 12, 13):
        docs = ds_splice_docs(seed)
        L.ygm_diag_read(dg.ctypes.data, 1)
        res = e.merge_updates_batch(docs)
        L.ygm_diag_read(dg.ctypes.data, 1)
        ok = [res[i] == oracle.merge_updates(us) for i, us in enumerate(docs)]
        print({"seed": seed, "parity": ok, "big_docs": int(dg[21]), "spliced": int(dg[22])}, flush=True)
    sys.exit(0)
C5 = os.environ.get("C5") == "1"   # C5-shaped documents (XmlFragment, 10 000 clients) instead of C3-shaped
for mb in ([float(x) for x in os.environ['BIG_MB'].split(',')] if os.environ.get('BIG_MB') else (0.3, 1, 3, 10)):
    if C5:
        arena, upd_off, doc_upd = synth.big_docs(1, int(mb * 1e6), 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
    else:
        arena, upd_off, doc_upd = synth.big_docs(1, int(mb * 1e6), 1024, max_clients=64, max_k=200, seed=8)
    n = 1
    upd_doc = np.zeros(len(upd_off) - 1, np.uint32)
    ms = []
    for rep in range(3):
        s0 = e.stats(); t0 = time.time()
        res = e.merge_packed(arena, upd_off, upd_doc, n)
        s1 = e.stats()
        ms.append((round(s1.kernel_ms - s0.kernel_ms, 2), round((time.time() - t0) * 1e3, 1)))
    st, out = oracle.merge_updates([bytes(arena[int(upd_off[i]):int(upd_off[i + 1])]) for i in range(len(upd_off) - 1)])
    ok = res[0] == (st, out)
    line = {"MB": mb, "bytes": int(upd_off[-1]), "updates": len(upd_off) - 1, "kernel_ms_and_wall_ms": ms, "docs_big": s1.docs_big, "parity": ok}
    if diag:
        L = eng.lib()
        L.ygm_diag_ts_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
        ts = np.zeros(16384 * 8, np.uint64)
        L.ygm_diag_ts_read(ts.ctypes.data, 0)
        L.ygm_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
        dg = np.zeros(32, np.uint64)
        L.ygm_diag_read(dg.ctypes.data, 1)
        line["ds_plan"] = {"big_docs": int(dg[21]), "spliced": int(dg[22]), "ds_values": int(dg[23]), "ds_entries": int(dg[24])}
        line["follow"] = {"blocks": int(dg[16]), "steps": int(dg[17]), "structs": int(dg[18]), "global": int(dg[19]), "hdr_slow": int(dg[20]),
                          "us_tile_hdr_structs_tail (all runs)": [int(dg[i]) / 100.0 for i in (25, 26, 27, 28)]}
        t = ts.reshape(16384, 8)[0].astype(np.int64)
        d = np.diff(t[:6]) * 10 / 1000.0
        if dsmode:   # slots 6 / 7: where each pass's delete-set part starts (absolute stamps)
            line["ds_us"] = {"pass0 structs": (t[6] - t[3]) * 10 / 1000.0, "pass0 ds": (t[4] - t[6]) * 10 / 1000.0,
                             "pass1 structs": (t[7] - t[4]) * 10 / 1000.0, "pass1 ds": (t[5] - t[7]) * 10 / 1000.0}
        line["phases_us"] = {"log walk": d[0], "U0 follow+spec+validate": d[1], "spec": t[6] * 10 / 1000.0, "validate": t[7] * 10 / 1000.0,
                             "sorts": d[2], "pass0": d[3], "pass1": d[4]}
    print(line, flush=True)
