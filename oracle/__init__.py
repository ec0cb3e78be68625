"""CPU oracle for the yjs update-level functions -- TEST INFRASTRUCTURE ONLY.

ctypes binding of ``liboracle.so`` (built from ``yjs_oracle.c`` by the Makefile
next to it).  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package; the product path
(``hocuspocus_amd``) never does.

Functions mirror yjs (13.6.26 semantics by default, ``compat135=True`` for the
13.5.16 fixtures):

* ``merge_updates(updates)``            -> ``Y.mergeUpdates``               (Y@39011)
* ``diff_update(update, sv)``           -> ``Y.diffUpdate``                 (Y@40711)
* ``encode_state_vector_from_update(u)``-> ``Y.encodeStateVectorFromUpdate`` (Y@37728)

Each returns ``(status, bytes|None)``; status 0 is success, otherwise one of
``STATUS_NAMES`` (yjs would throw, or the content would be re-encoded).
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

STATUS_NAMES = {0: "OK", 1: "EMALFORMED", 2: "ERANGE", 3: "ENONCANON", 4: "ESURROGATE", 5: "EDEPTH", 6: "ENOMEM"}
COMPAT_135 = 1
KEEP_SUB = 4    # diff: keep each struct's parentSub bit (YO_KEEP_SUB)

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "yjs_oracle.c")):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        u8p = P(ctypes.c_uint8)
        L.yo_merge.argtypes = [P(u8p), P(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int, P(u8p), P(ctypes.c_size_t)]
        L.yo_diff.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_int, P(u8p), P(ctypes.c_size_t)]
        L.yo_sv.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, P(u8p), P(ctypes.c_size_t)]
        L.yo_free.argtypes = [ctypes.c_void_p]
        L.yo_merge_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        L.yo_doc_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        L.yo_v8_sort_table.argtypes = [P(ctypes.c_int), ctypes.c_int, P(ctypes.c_int8)]
        L.yo_v8_sort_table.restype = ctypes.c_long
        for f in (L.yo_merge, L.yo_diff, L.yo_sv):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def _buf(b):
    b = bytes(b)
    arr = (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(b if b else b"\0")
    return arr, len(b)


def _take(out, n, st):
    L = lib()
    try:
        if st != 0:
            return st, None
        return 0, ctypes.string_at(out, n.value)
    finally:
        if out:
            L.yo_free(out)


def merge_updates(updates, compat135=False):
    L = lib()
    bufs = [_buf(u) for u in updates]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(n, 1))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(n, 1))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_merge(ptrs, lens, n, COMPAT_135 if compat135 else 0, ctypes.byref(out), ctypes.byref(olen))
    return _take(out, olen, st)


def diff_update(update, sv, compat135=False, keep_sub=False):
    """yjs diffUpdate(update, sv); keep_sub: every struct keeps its input's parentSub bit (encodeStateAsUpdate(doc, sv)
    of a document loaded from `update` when `update` is that document's own encodeStateAsUpdate)."""
    L = lib()
    ub, ul = _buf(update)
    sb, sl = _buf(sv)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_diff(ctypes.cast(ub, ctypes.POINTER(ctypes.c_uint8)), ul, ctypes.cast(sb, ctypes.POINTER(ctypes.c_uint8)), sl,
                   (COMPAT_135 if compat135 else 0) | (KEEP_SUB if keep_sub else 0), ctypes.byref(out), ctypes.byref(olen))
    return _take(out, olen, st)


def encode_state_vector_from_update(update, compat135=False):
    L = lib()
    ub, ul = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_sv(ctypes.cast(ub, ctypes.POINTER(ctypes.c_uint8)), ul, COMPAT_135 if compat135 else 0, ctypes.byref(out), ctypes.byref(olen))
    return _take(out, olen, st)


def v8_sort_table(arr, table):
    """Sort ids `arr` the way V8's Array.prototype.sort does with comparator table[a*n+b]."""
    L = lib()
    n = len(arr)
    a = (ctypes.c_int * max(n, 1))(*arr)
    t = (ctypes.c_int8 * max(len(table), 1))(*table)
    calls = L.yo_v8_sort_table(a, n, t)
    return list(a)[:n], calls


def merge_batch(arena, upd_off, doc_upd, threads=1, compat135=False):
    """mergeUpdates over every document of a packed corpus on `threads` pthreads
    (CPU-baseline driver).  Returns (status int32 array, algorithmic bytes)."""
    import numpy as np
    L = lib()
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    upd_off = np.ascontiguousarray(upd_off, dtype=np.uint64)
    doc_upd = np.ascontiguousarray(doc_upd, dtype=np.uint32)
    n_docs = len(doc_upd) - 1
    status = np.zeros(max(n_docs, 1), dtype=np.int32)
    algo = ctypes.c_uint64()
    L.yo_merge_batch(arena.ctypes.data, upd_off.ctypes.data, doc_upd.ctypes.data, n_docs, COMPAT_135 if compat135 else 0,
                     threads, status.ctypes.data, ctypes.byref(algo))
    return status[:n_docs], algo.value


def doc_batch(mode, arena, doc_off, sv_arena=None, sv_off=None, threads=1, compat135=False):
    """encodeStateVectorFromUpdate (mode "sv") or diffUpdate (mode "diff") over every document of a
    packed corpus on `threads` pthreads (CPU-baseline driver).  Returns (status int32 array, algorithmic bytes)."""
    import numpy as np
    L = lib()
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
    n_docs = len(doc_off) - 1
    if mode == "diff":
        sv_arena = np.ascontiguousarray(sv_arena, dtype=np.uint8)
        sv_off = np.ascontiguousarray(sv_off, dtype=np.uint64)
    status = np.zeros(max(n_docs, 1), dtype=np.int32)
    algo = ctypes.c_uint64()
    L.yo_doc_batch(1 if mode == "diff" else 0, arena.ctypes.data, doc_off.ctypes.data,
                   sv_arena.ctypes.data if mode == "diff" else None, sv_off.ctypes.data if mode == "diff" else None,
                   n_docs, COMPAT_135 if compat135 else 0, threads, status.ctypes.data, ctypes.byref(algo))
    return status[:n_docs], algo.value


# ---- update V2 (yjs_oracle_v2.c) ----
def _v2lib():
    L = lib()
    if not getattr(L, "_v2", False):
        P = ctypes.POINTER
        u8p = P(ctypes.c_uint8)
        L.yo_merge_v2.argtypes = [P(u8p), P(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int, P(u8p), P(ctypes.c_size_t)]
        L.yo_diff_v2.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_int, P(u8p), P(ctypes.c_size_t)]
        for f in (L.yo_sv_v2, L.yo_v1_to_v2, L.yo_v2_to_v1):
            f.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, P(u8p), P(ctypes.c_size_t)]
        for f in (L.yo_merge_v2, L.yo_diff_v2, L.yo_sv_v2, L.yo_v1_to_v2, L.yo_v2_to_v1):
            f.restype = ctypes.c_int
        L._v2 = True
    return L


def merge_updates_v2(updates, compat135=False):
    """Y.mergeUpdatesV2 (V2 in, V2 out)."""
    L = _v2lib()
    bufs = [_buf(u) for u in updates]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(n, 1))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(n, 1))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_merge_v2(ptrs, lens, n, COMPAT_135 if compat135 else 0, ctypes.byref(out), ctypes.byref(olen))
    return _take(out, olen, st)


def diff_update_v2(update, sv, compat135=False):
    """Y.diffUpdateV2 (V2 update, V1-format state vector)."""
    L = _v2lib()
    ub, ul = _buf(update)
    sb, sl = _buf(sv)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_diff_v2(ctypes.cast(ub, ctypes.POINTER(ctypes.c_uint8)), ul, ctypes.cast(sb, ctypes.POINTER(ctypes.c_uint8)), sl,
                      COMPAT_135 if compat135 else 0, ctypes.byref(out), ctypes.byref(olen))
    return _take(out, olen, st)


def _unary_v2(fn, update, compat135):
    L = _v2lib()
    ub, ul = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = getattr(L, fn)(ctypes.cast(ub, ctypes.POINTER(ctypes.c_uint8)), ul, COMPAT_135 if compat135 else 0, ctypes.byref(out),
                        ctypes.byref(olen))
    return _take(out, olen, st)


def encode_state_vector_from_update_v2(update, compat135=False):
    """Y.encodeStateVectorFromUpdateV2."""
    return _unary_v2("yo_sv_v2", update, compat135)


def convert_update_format_v1_to_v2(update, compat135=False):
    """yjs 13.6 convertUpdateFormatV1ToV2."""
    return _unary_v2("yo_v1_to_v2", update, compat135)


def convert_update_format_v2_to_v1(update, compat135=False):
    """yjs 13.6 convertUpdateFormatV2ToV1 (Any numbers that are not varInt integers in embeds / formats are refused)."""
    return _unary_v2("yo_v2_to_v1", update, compat135)
