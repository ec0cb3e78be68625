"""Seeded synthetic Yjs update-v1 corpora (ctypes over tools/libsynth.so).

Bench / test infrastructure: the GPU box has no yjs, so corpora are emitted as
V1 bytes directly.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libsynth.so")
        if not os.path.exists(path) or os.path.getmtime(path) < max(os.path.getmtime(os.path.join(_HERE, f)) for f in ("synth.c", "synth_live.c")):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.synth_text_updates.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P, P, P,
                                         ctypes.c_int]
        L.synth_text_updates.restype = ctypes.c_size_t
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.synth_text_states_gen.argtypes = [ctypes.c_uint64, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, u64p, u64p]
        L.synth_text_updates_gen.argtypes = [ctypes.c_uint64, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_int, ctypes.c_uint32, u64p, u64p]
        L.synth_text_updates_gen.restype = P
        L.synth_text_updates_take.argtypes = [P, P, P, P]
        L.synth_text_updates_take.restype = None
        L.synth_partition.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, P]
        L.synth_partition.restype = ctypes.c_uint32
        L.synth_text_states_gen.restype = P
        L.synth_text_states_take.argtypes = [P, P, P, P, P]
        L.synth_text_states_take.restype = None
        L.synth_live_docs.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_int, P, P, P]
        L.synth_live_docs.restype = ctypes.c_size_t
        L.synth_big_docs.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_int, P, P, P]
        L.synth_big_docs.restype = ctypes.c_size_t
        _lib = L
    return _lib


def text_updates(n_docs, n_updates=200, min_clients=1, max_clients=4, del_pct=0, seed=1, max_run=1):
    """Config C2: returns (arena uint8, upd_off uint64[n_upd+1], doc_upd uint32[n_docs+1]).  max_run > 1: each
    insert is one Item of 1..max_run characters (pastes, words typed in one transaction)."""
    n_upd = n_docs * n_updates
    buf = np.empty(n_upd * (40 + max_run) + 64, dtype=np.uint8)
    upd_off = np.empty(n_upd + 1, dtype=np.uint64)
    doc_upd = np.empty(n_docs + 1, dtype=np.uint32)
    n = lib().synth_text_updates(seed, n_docs, n_updates, min_clients, max_clients, del_pct,
                                 buf.ctypes.data, upd_off.ctypes.data, doc_upd.ctypes.data, max_run)
    return buf[:n].copy(), upd_off, doc_upd


def _threads(threads):
    return threads if threads else max(1, min(16, len(os.sched_getaffinity(0))))


def partition(prefix, n_total, world, rank):
    """Global indices of the documents named prefix + str(i), i < n_total, that rank owns:
    fnv1a64(name) mod world (hocuspocus_amd.shard.shard_of)."""
    out = np.empty(max(n_total, 1), dtype=np.uint32)
    k = lib().synth_partition(prefix.encode(), n_total, world, rank, out.ctypes.data)
    return out[:k].copy()


def text_updates_docs(idx, n_updates=200, min_clients=1, max_clients=4, del_pct=0, seed=1, threads=None):
    """Config C2 for the documents of global indices `idx` (each from its own PRNG stream: a rank's shard
    is generated alone).  Returns (arena, upd_off[n_upd+1], doc_upd[n+1])."""
    idx = np.ascontiguousarray(idx, dtype=np.uint32)
    n = len(idx)
    nb, nu = ctypes.c_uint64(), ctypes.c_uint64()
    h = lib().synth_text_updates_gen(seed, idx.ctypes.data, n, n_updates, min_clients, max_clients, del_pct, _threads(threads),
                                     ctypes.byref(nb), ctypes.byref(nu))
    buf = np.empty(nb.value, dtype=np.uint8)
    upd_off = np.empty(nu.value + 1, dtype=np.uint64)
    doc_upd = np.empty(n + 1, dtype=np.uint32)
    lib().synth_text_updates_take(h, buf.ctypes.data, upd_off.ctypes.data, doc_upd.ctypes.data)
    return buf, upd_off, doc_upd


def text_states(n_docs, min_bytes=1024, max_bytes=8192, min_clients=1, max_clients=16, seed=1, threads=None, idx=None):
    """Config C4: merged Y.Text states of 1-16 clients, log-uniform 1-8 KB, plus one
    state vector per document.  Returns (arena, doc_off[n_docs+1], sv_arena, sv_off[n_docs+1]).
    Documents come from per-document PRNG streams (global index i, or idx[i]), so the bytes do not
    depend on `threads` and a rank's shard is generated alone."""
    if idx is not None:
        idx = np.ascontiguousarray(idx, dtype=np.uint32)
        n_docs = len(idx)
    nb, ns = ctypes.c_uint64(), ctypes.c_uint64()
    h = lib().synth_text_states_gen(seed, idx.ctypes.data if idx is not None else None, n_docs, min_bytes, max_bytes, min_clients,
                                    max_clients, _threads(threads), ctypes.byref(nb), ctypes.byref(ns))
    buf = np.empty(nb.value, dtype=np.uint8)
    sv = np.empty(ns.value, dtype=np.uint8)
    doc_off = np.empty(n_docs + 1, dtype=np.uint64)
    sv_off = np.empty(n_docs + 1, dtype=np.uint64)
    lib().synth_text_states_take(h, buf.ctypes.data, doc_off.ctypes.data, sv.ctypes.data, sv_off.ctypes.data)
    return buf, doc_off, sv, sv_off


def big_docs(n_docs, max_bytes, min_bytes=1024, max_clients=64, max_k=200, xml=False, seed=1):
    """Configs C3 / C5: [snapshot, ...log] per document, snapshot of max_bytes * rank^-0.8 bytes
    (C3: GC / deleted content / strings, a merged delete set, 40 % deletions in the log; C5 with
    xml=True and max_clients=10000: XmlElement / XmlText / ContentFormat / ContentEmbed runs over
    thousands of client blocks).  Returns (arena, upd_off[n_upd+1], doc_upd[n_docs+1])."""
    sizes = np.maximum(max_bytes * np.arange(1, n_docs + 1, dtype=np.float64) ** -0.8, min_bytes)
    cap = int(sizes.sum() * 1.6) + n_docs * (max_clients * 512 + max_k * 64 + 4096)
    buf = np.empty(cap, dtype=np.uint8)
    upd_off = np.empty(n_docs * max_k + 1, dtype=np.uint64)
    doc_upd = np.empty(n_docs + 1, dtype=np.uint32)
    n = lib().synth_big_docs(seed, n_docs, int(max_bytes), int(min_bytes), max_clients, max_k, 1 if xml else 0,
                             buf.ctypes.data, upd_off.ctypes.data, doc_upd.ctypes.data)
    assert n <= cap
    nu = int(doc_upd[n_docs])
    return buf[:n].copy(), upd_off[:nu + 1].copy(), doc_upd


def live_docs(n_docs, max_bytes, min_bytes=1024, n_clients=64, max_k=200, xml=False, seed=1, threads=None):
    """f-1 at BASELINE sizes (tools/synth_live.c): [state, ...log] documents of a simulated Y.Doc session that
    Y.applyUpdate integrates completely -- xml=True: Tiptap-style XmlFragment (paragraphs, XmlText runs, formats,
    embeds, attributes; n_clients > 64: exactly that many client blocks, config C5), else one Y.Text with heavy
    deletions (config C3's shape).  State of max_bytes * rank^-0.8 bytes.  Documents come from per-document PRNG
    streams, generated in chunks on threads (ctypes releases the GIL).  Returns (arena, upd_off, doc_upd)."""
    from concurrent.futures import ThreadPoolExecutor
    L = lib()
    nt = max(1, min(_threads(threads), n_docs))
    bounds = [n_docs * t // nt for t in range(nt + 1)]

    def part(t):
        d0, d1 = bounds[t], bounds[t + 1]
        m = d1 - d0
        sizes = np.maximum(max_bytes * np.arange(d0 + 1, d1 + 1, dtype=np.float64) ** -0.8, min_bytes)
        cap = int(sizes.sum() * 2.0) + m * (max_k * 160 + (n_clients * 64 if xml else 0) + 65536)
        buf = np.empty(cap, dtype=np.uint8)
        uo = np.empty(m * max_k + 1, dtype=np.uint64)
        du = np.empty(m + 1, dtype=np.uint32)
        n = L.synth_live_docs(seed, d0, m, int(max_bytes), int(min_bytes), n_clients, max_k, 1 if xml else 0,
                              buf.ctypes.data, uo.ctypes.data, du.ctypes.data)
        assert n <= cap
        return buf[:n], uo[:int(du[-1]) + 1], du
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(part, range(nt)))
    arena = np.concatenate([p[0] for p in parts])
    upd_off, doc_upd, b, u = [], [], 0, 0
    for buf, uo, du in parts:
        upd_off.append(uo[:-1] + np.uint64(b))
        doc_upd.append(du[:-1] + np.uint32(u))
        b += len(buf)
        u += int(du[-1])
    upd_off.append(np.array([b], np.uint64))
    doc_upd.append(np.array([u], np.uint32))
    return arena, np.concatenate(upd_off), np.concatenate(doc_upd)


def split(arena, off):
    """bytes objects of each [off[i], off[i+1]) slice."""
    a = arena.tobytes()
    o = [int(x) for x in off]
    return [a[o[i]:o[i + 1]] for i in range(len(o) - 1)]
