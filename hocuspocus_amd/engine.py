"""ctypes binding of libygm.so (include/ygm.h) -- the MI355X batched Yjs update engine.

Python mirror of the yjs update-level API that Hocuspocus's persistence and
sync path calls, batched over documents:

* ``Engine.merge_updates_batch(docs)``          per document ``Y.mergeUpdates(updates)``
* ``Engine.diff_update_batch(updates, svs)``    per document ``Y.diffUpdate(update, sv)``
* ``Engine.encode_state_vector_from_update_batch(updates)``
                                                 per document ``Y.encodeStateVectorFromUpdate``

Single-document helpers (``merge_updates`` ...) raise :class:`YjsError` where yjs
throws, mirroring the reference's error behaviour.  There is no CPU fallback:
if the HIP library is missing or no GPU is present, construction fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YGM_LIB") or os.path.join(_HERE, "libygm.so")  # YGM_LIB: experiment builds (tooling)

OK, EMALFORMED, ERANGE, ENONCANON, ESURROGATE, EDEPTH, ENOMEM, EDEVICE, EINVAL, EUNSUPPORTED = range(10)
STATUS_NAMES = {0: "OK", 1: "EMALFORMED", 2: "ERANGE", 3: "ENONCANON", 4: "ESURROGATE", 5: "EDEPTH",
                6: "ENOMEM", 7: "EDEVICE", 8: "EINVAL", 9: "EUNSUPPORTED"}
F_COMPAT_135 = 1
F_FORCE_SEQ = 2


class YjsError(Exception):
    """Raised where yjs would throw (or where the engine refuses a document)."""

    def __init__(self, code: int):
        self.code = code
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {strerror(code)}")


class _Result(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("off", ctypes.POINTER(ctypes.c_uint64)),
                ("len", ctypes.POINTER(ctypes.c_uint64)), ("status", ctypes.POINTER(ctypes.c_int32)),
                ("n_docs", ctypes.c_uint32), ("data_bytes", ctypes.c_uint64)]


class _DevResult(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("off", ctypes.c_void_p), ("len", ctypes.c_void_p),
                ("status", ctypes.c_void_p), ("data_bytes", ctypes.c_uint64), ("payload_bytes", ctypes.c_uint64)]


class Stats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("docs", ctypes.c_uint64), ("updates", ctypes.c_uint64),
                ("bytes_in", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64), ("docs_fast", ctypes.c_uint64),
                ("docs_seq", ctypes.c_uint64), ("kernel_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double),
                ("docs_lean", ctypes.c_uint64), ("lean_ms", ctypes.c_double),
                ("lean_launches", ctypes.c_uint64), ("docs_big", ctypes.c_uint64),
                ("docs_lean_wide", ctypes.c_uint64), ("host_syncs", ctypes.c_uint64),
                ("docs_pending", ctypes.c_uint64)]


_lib = None

# every symbol include/ygm.h declares
EXPORTS = ("ygm_open", "ygm_close", "ygm_merge_v1", "ygm_diff_v1", "ygm_sv_from_update_v1", "ygm_merge_v1_device",
           "ygm_merge_v1_device_async", "ygm_merge_v1_device_finish",
           "ygm_diff_v1_device", "ygm_sv_from_update_v1_device", "ygm_snapshot_v1", "ygm_snapshot_v1_device",
           "ygm_contains_v1", "ygm_contains_v1_device", "ygm_stats", "ygm_strerror", "ygm_version",
           "ygm_merge_v2", "ygm_diff_v2", "ygm_sv_from_update_v2", "ygm_convert_v1_to_v2", "ygm_convert_v2_to_v1",
           "ygm_merge_v2_device", "ygm_diff_v2_device", "ygm_sv_from_update_v2_device", "ygm_convert_v1_to_v2_device",
           "ygm_convert_v2_to_v1_device", "ygm_sync_step2_v1", "ygm_sync_step2_v1_device",
           "ygm_merge_v1_device_lens", "ygm_merge_v1_device_lens_async")


def lib():
    """Loads libygm.so (raises OSError when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: the torch wheel bundles its own libamdhip64.so.7 (same soname as
        # /opt/rocm's).  Whichever loads first serves both, and torch's CUDA init fails ("No HIP GPUs are
        # available") on the system copy -- so when torch is installed it loads first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        L.ygm_open.argtypes = [ctypes.c_int, u32, ctypes.POINTER(vp)]
        L.ygm_close.argtypes = [vp]
        L.ygm_close.restype = None
        L.ygm_merge_v1.argtypes = [vp, vp, vp, vp, u32, u32, ctypes.POINTER(_Result)]
        L.ygm_diff_v1.argtypes = [vp, vp, vp, vp, vp, u32, ctypes.POINTER(_Result)]
        L.ygm_sv_from_update_v1.argtypes = [vp, vp, vp, u32, ctypes.POINTER(_Result)]
        L.ygm_merge_v1_device.argtypes = [vp, vp, u64, vp, vp, u32, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_merge_v1_device_async.argtypes = [vp, vp, u64, vp, vp, u32, u32, vp]
        L.ygm_merge_v1_device_finish.argtypes = [vp, ctypes.POINTER(_DevResult)]
        L.ygm_merge_v1_device_lens.argtypes = [vp, vp, u64, vp, vp, vp, u32, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_merge_v1_device_lens_async.argtypes = [vp, vp, u64, vp, vp, vp, u32, u32, vp]
        L.ygm_diff_v1_device.argtypes = [vp, vp, u64, vp, vp, vp, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_sv_from_update_v1_device.argtypes = [vp, vp, u64, vp, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_snapshot_v1.argtypes = [vp, vp, vp, u32, ctypes.POINTER(_Result)]
        L.ygm_snapshot_v1_device.argtypes = [vp, vp, u64, vp, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_contains_v1.argtypes = [vp, vp, vp, vp, vp, u32, ctypes.POINTER(_Result)]
        L.ygm_contains_v1_device.argtypes = [vp, vp, vp, vp, vp, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_sync_step2_v1.argtypes = [vp, vp, vp, vp, vp, u32, ctypes.POINTER(_Result)]
        L.ygm_sync_step2_v1_device.argtypes = [vp, vp, u64, vp, vp, vp, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_merge_v2.argtypes = [vp, vp, vp, vp, u32, u32, ctypes.POINTER(_Result)]
        L.ygm_diff_v2.argtypes = [vp, vp, vp, vp, vp, u32, ctypes.POINTER(_Result)]
        for f in ("ygm_sv_from_update_v2", "ygm_convert_v1_to_v2", "ygm_convert_v2_to_v1"):
            getattr(L, f).argtypes = [vp, vp, vp, u32, ctypes.POINTER(_Result)]
        L.ygm_merge_v2_device.argtypes = [vp, vp, u64, vp, vp, u32, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_diff_v2_device.argtypes = [vp, vp, u64, vp, vp, vp, u32, vp, ctypes.POINTER(_DevResult)]
        for f in ("ygm_sv_from_update_v2_device", "ygm_convert_v1_to_v2_device", "ygm_convert_v2_to_v1_device"):
            getattr(L, f).argtypes = [vp, vp, u64, vp, u32, vp, ctypes.POINTER(_DevResult)]
        L.ygm_stats.argtypes = [vp, ctypes.POINTER(Stats)]
        L.ygm_strerror.argtypes = [i32]
        L.ygm_strerror.restype = ctypes.c_char_p
        L.ygm_version.restype = ctypes.c_char_p
        for f in ("ygm_open", "ygm_merge_v1", "ygm_diff_v1", "ygm_sv_from_update_v1", "ygm_merge_v1_device",
                  "ygm_merge_v1_device_async", "ygm_merge_v1_device_finish",
                  "ygm_diff_v1_device", "ygm_sv_from_update_v1_device", "ygm_snapshot_v1", "ygm_snapshot_v1_device",
                  "ygm_contains_v1", "ygm_contains_v1_device", "ygm_stats", "ygm_merge_v2", "ygm_diff_v2", "ygm_sv_from_update_v2",
                  "ygm_convert_v1_to_v2", "ygm_convert_v2_to_v1", "ygm_merge_v2_device", "ygm_diff_v2_device",
                  "ygm_sv_from_update_v2_device", "ygm_convert_v1_to_v2_device", "ygm_convert_v2_to_v1_device",
                  "ygm_sync_step2_v1", "ygm_sync_step2_v1_device", "ygm_merge_v1_device_lens", "ygm_merge_v1_device_lens_async"):
            getattr(L, f).restype = i32
        _lib = L
    return _lib


def strerror(code: int) -> str:
    return lib().ygm_strerror(code).decode()


def _pack(blobs):
    arena = b"".join(blobs)
    off = np.zeros(len(blobs) + 1, dtype=np.uint64)
    if blobs:
        np.cumsum(np.fromiter((len(b) for b in blobs), dtype=np.uint64, count=len(blobs)), out=off[1:])
    return arena, off


def _ptr(a):
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_char_p(a) if a else None


TAIL_PAD = 64   # readable bytes the kernels need after a device arena (include/ygm.h, "Tail padding")


def _dptr(x, need=0):
    """A device pointer: an int, or a tensor (then its allocation must hold `need` bytes)."""
    if hasattr(x, "data_ptr"):
        nbytes = x.numel() * x.element_size()
        if nbytes < need:
            raise ValueError(f"device buffer of {nbytes} bytes: the engine reads {need} (arena + {TAIL_PAD} bytes of tail padding)")
        return x.data_ptr()
    return int(x)


@dataclass
class DeviceResult:
    """Outputs left in HBM by a device-resident call (context-owned memory)."""
    data: int
    off: int
    len: int
    status: int
    data_bytes: int      # used extent of `data` (merge outputs sit in per-document slots)
    payload_bytes: int   # sum of the per-document output lengths


class Engine:
    """One engine context on one GPU (not thread-safe; one batch in flight)."""

    def __init__(self, device: int = 0, compat135: bool = False, force_seq: bool = False):
        flags = (F_COMPAT_135 if compat135 else 0) | (F_FORCE_SEQ if force_seq else 0)
        ctx = ctypes.c_void_p()
        st = lib().ygm_open(device, flags, ctypes.byref(ctx))
        if st != OK:
            raise YjsError(st)
        self._ctx = ctx
        self.device = device

    def close(self):
        if getattr(self, "_ctx", None):
            lib().ygm_close(self._ctx)
            self._ctx = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------ results
    @staticmethod
    def _unpack(res: _Result):
        n = res.n_docs
        if n == 0:
            return []
        off = np.ctypeslib.as_array(res.off, shape=(n,))
        ln = np.ctypeslib.as_array(res.len, shape=(n,))
        status = np.ctypeslib.as_array(res.status, shape=(n,))
        data = ctypes.string_at(res.data, res.data_bytes) if res.data_bytes else b""
        out = []
        for d in range(n):
            st = int(status[d])
            if st == OK:
                o = int(off[d])
                out.append((OK, data[o:o + int(ln[d])]))
            else:
                out.append((st, None))
        return out

    # ------------------------------------------------------------ batch API
    def merge_updates_batch(self, docs):
        """docs: list of lists of update bytes -> list of (status, merged bytes | None)."""
        blobs, doc_ids = [], []
        for d, ups in enumerate(docs):
            for u in ups:
                blobs.append(bytes(u))
                doc_ids.append(d)
        arena, off = _pack(blobs)
        upd_doc = np.asarray(doc_ids, dtype=np.uint32)
        res = _Result()
        st = lib().ygm_merge_v1(self._ctx, arena or None, _ptr(off), _ptr(upd_doc), len(blobs), len(docs), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    def merge_packed(self, arena: np.ndarray, upd_off: np.ndarray, upd_doc: np.ndarray, n_docs: int):
        """Packed host-array form of merge_updates_batch (arena uint8, upd_off uint64, upd_doc uint32)."""
        res = _Result()
        st = lib().ygm_merge_v1(self._ctx, _ptr(arena), _ptr(upd_off), _ptr(upd_doc), len(upd_doc), n_docs, ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    @staticmethod
    def _raw(res: _Result):
        n = res.n_docs
        if n == 0:
            return (np.zeros(0, np.int32), np.zeros(0, np.uint64), np.zeros(0, np.uint64), b"")
        return (np.ctypeslib.as_array(res.status, shape=(n,)), np.ctypeslib.as_array(res.off, shape=(n,)),
                np.ctypeslib.as_array(res.len, shape=(n,)), (ctypes.c_uint8 * max(res.data_bytes, 1)).from_address(ctypes.cast(res.data, ctypes.c_void_p).value))

    def merge_packed_raw(self, arena: np.ndarray, upd_off: np.ndarray, upd_doc: np.ndarray, n_docs: int):
        """merge_packed without the per-document Python unpacking: (status, off, len, data) views of the
        context's pinned result buffers, valid until the next call on this engine."""
        res = _Result()
        st = lib().ygm_merge_v1(self._ctx, _ptr(arena), _ptr(upd_off), _ptr(upd_doc), len(upd_doc), n_docs, ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._raw(res)

    def doc_packed_raw(self, op: str, arena: np.ndarray, doc_off: np.ndarray, sv_arena=None, sv_off=None):
        """Host-array SV ("sv") / diff ("diff") batch; result views as merge_packed_raw."""
        res = _Result()
        n = len(doc_off) - 1
        if op == "diff":
            st = lib().ygm_diff_v1(self._ctx, _ptr(arena), _ptr(doc_off), _ptr(sv_arena), _ptr(sv_off), n, ctypes.byref(res))
        else:
            st = lib().ygm_sv_from_update_v1(self._ctx, _ptr(arena), _ptr(doc_off), n, ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._raw(res)

    def diff_update_batch(self, updates, svs):
        arena, off = _pack([bytes(u) for u in updates])
        sva, svo = _pack([bytes(s) for s in svs])
        res = _Result()
        st = lib().ygm_diff_v1(self._ctx, arena or None, _ptr(off), sva or None, _ptr(svo), len(updates), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    def encode_state_vector_from_update_batch(self, updates):
        arena, off = _pack([bytes(u) for u in updates])
        res = _Result()
        st = lib().ygm_sv_from_update_v1(self._ctx, arena or None, _ptr(off), len(updates), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    # ------------------------------------------------------------ update V2
    def merge_updates_v2_batch(self, docs):
        """Y.mergeUpdatesV2 per document: docs = list of lists of V2 updates -> list of (status, V2 bytes | None)."""
        blobs, doc_ids = [], []
        for d, ups in enumerate(docs):
            for u in ups:
                blobs.append(bytes(u))
                doc_ids.append(d)
        arena, off = _pack(blobs)
        upd_doc = np.asarray(doc_ids, dtype=np.uint32)
        res = _Result()
        st = lib().ygm_merge_v2(self._ctx, arena or None, _ptr(off), _ptr(upd_doc), len(blobs), len(docs), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    def diff_update_v2_batch(self, updates, svs):
        """Y.diffUpdateV2(update, sv) per document (V2 updates, V1-format state vectors)."""
        arena, off = _pack([bytes(u) for u in updates])
        sva, svo = _pack([bytes(s) for s in svs])
        res = _Result()
        st = lib().ygm_diff_v2(self._ctx, arena or None, _ptr(off), sva or None, _ptr(svo), len(updates), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    def _unary_v2(self, fn, updates):
        arena, off = _pack([bytes(u) for u in updates])
        res = _Result()
        st = getattr(lib(), fn)(self._ctx, arena or None, _ptr(off), len(updates), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    def _conv_packed(self, fn, arena, doc_off):
        """Packed host-array form of a unary V2 call (ygm_sv_from_update_v2 / ygm_convert_*): the raw _Result."""
        res = _Result()
        st = getattr(lib(), fn)(self._ctx, _ptr(arena), _ptr(doc_off), len(doc_off) - 1, ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return res

    def encode_state_vector_from_update_v2_batch(self, updates):
        """Y.encodeStateVectorFromUpdateV2 per update (the state vector is V1-encoded, as yjs's)."""
        return self._unary_v2("ygm_sv_from_update_v2", updates)

    def convert_update_format_v1_to_v2_batch(self, updates):
        """yjs 13.6 Y.convertUpdateFormatV1ToV2 per update."""
        return self._unary_v2("ygm_convert_v1_to_v2", updates)

    def convert_update_format_v2_to_v1_batch(self, updates):
        """yjs 13.6 Y.convertUpdateFormatV2ToV1 per update."""
        return self._unary_v2("ygm_convert_v2_to_v1", updates)

    def merge_v2_device(self, d_arena, arena_bytes, d_upd_off, d_doc_upd, n_upd, n_docs, stream=0) -> "DeviceResult":
        r = _DevResult()
        st = lib().ygm_merge_v2_device(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_upd_off), _dptr(d_doc_upd),
                                       n_upd, n_docs, stream or None, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    def doc_v2_device(self, op, d_arena, arena_bytes, d_doc_off, n_docs, d_sv=None, d_sv_off=None, stream=0) -> "DeviceResult":
        """op: "diff" (d_sv / d_sv_off), "sv", "v1_to_v2", "v2_to_v1" -- the device-resident V2 calls."""
        r = _DevResult()
        a = _dptr(d_arena, arena_bytes + TAIL_PAD)
        if op == "diff":
            st = lib().ygm_diff_v2_device(self._ctx, a, arena_bytes, _dptr(d_doc_off), _dptr(d_sv), _dptr(d_sv_off), n_docs, stream or None,
                                          ctypes.byref(r))
        else:
            fn = {"sv": "ygm_sv_from_update_v2_device", "v1_to_v2": "ygm_convert_v1_to_v2_device",
                  "v2_to_v1": "ygm_convert_v2_to_v1_device"}[op]
            st = getattr(lib(), fn)(self._ctx, a, arena_bytes, _dptr(d_doc_off), n_docs, stream or None, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    # ------------------------------------------------------------ yjs-shaped single calls
    def snapshot_batch(self, updates):
        """Doc-normalized snapshots: Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), u)) per update
        (ygm_snapshot_v1) -> list of (status, bytes | None); UNSUPPORTED marks documents outside the envelope."""
        arena, off = _pack([bytes(u) for u in updates])
        res = _Result()
        st = lib().ygm_snapshot_v1(self._ctx, arena or None, _ptr(off), len(updates), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    def sync_step2_batch(self, states, svs):
        """SyncStep2 payloads of stored documents: Y.encodeStateAsUpdate(doc, sv) for doc = Y.applyUpdate(new Y.Doc(),
        state) (MessageReceiver.ts:137-138; ygm_sync_step2_v1) -> list of (status, bytes | None); UNSUPPORTED marks
        documents outside the snapshot envelope."""
        sa, so = _pack([bytes(s) for s in states])
        va, vo = _pack([bytes(v) for v in svs])
        res = _Result()
        st = lib().ygm_sync_step2_v1(self._ctx, sa or None, _ptr(so), va or None, _ptr(vo), len(states), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return self._unpack(res)

    def contains_batch(self, states, updates):
        """Read-only SyncStep2: Y.snapshotContainsUpdate(Y.snapshot(doc), update) per pair, `states` being the
        documents' normalized states (snapshot_batch) -> list of (status, bool | None)."""
        sa, so = _pack([bytes(s) for s in states])
        ua, uo = _pack([bytes(u) for u in updates])
        res = _Result()
        st = lib().ygm_contains_v1(self._ctx, sa or None, _ptr(so), ua or None, _ptr(uo), len(states), ctypes.byref(res))
        if st != OK:
            raise YjsError(st)
        return [(s, None if s != OK else b == b"\x01") for s, b in self._unpack(res)]

    def snapshot_device(self, d_arena, arena_bytes, d_doc_off, n_docs, stream=0) -> "DeviceResult":
        r = _DevResult()
        st = lib().ygm_snapshot_v1_device(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_doc_off), n_docs,
                                          stream or None, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    def merge_updates(self, updates):
        st, out = self.merge_updates_batch([list(updates)])[0]
        if st != OK:
            raise YjsError(st)
        return out

    def diff_update(self, update, sv):
        st, out = self.diff_update_batch([update], [sv])[0]
        if st != OK:
            raise YjsError(st)
        return out

    def encode_state_vector_from_update(self, update):
        st, out = self.encode_state_vector_from_update_batch([update])[0]
        if st != OK:
            raise YjsError(st)
        return out

    # ------------------------------------------------------------ device-resident API
    def merge_device(self, d_arena: int, arena_bytes: int, d_upd_off: int, d_doc_upd: int, n_upd: int, n_docs: int,
                     stream: int = 0) -> DeviceResult:
        r = _DevResult()
        st = lib().ygm_merge_v1_device(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_upd_off), _dptr(d_doc_upd),
                                       n_upd, n_docs, stream or None, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    def merge_device_async(self, d_arena: int, arena_bytes: int, d_upd_off: int, d_doc_upd: int, n_upd: int, n_docs: int,
                           stream: int = 0) -> None:
        """Enqueues a device-resident batch merge without waiting (ygm_merge_v1_device_async)."""
        st = lib().ygm_merge_v1_device_async(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_upd_off),
                                             _dptr(d_doc_upd), n_upd, n_docs, stream or None)
        if st != OK:
            raise YjsError(st)

    def merge_device_lens(self, d_arena: int, arena_bytes: int, d_doc_off: int, d_upd_len: int, d_doc_upd: int, n_upd: int,
                          n_docs: int, stream: int = 0) -> DeviceResult:
        """The compact input form (ygm_merge_v1_device_lens): u64 offset per document, u16 length per update."""
        r = _DevResult()
        st = lib().ygm_merge_v1_device_lens(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_doc_off),
                                            _dptr(d_upd_len), _dptr(d_doc_upd), n_upd, n_docs, stream or None, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    def merge_device_lens_async(self, d_arena: int, arena_bytes: int, d_doc_off: int, d_upd_len: int, d_doc_upd: int, n_upd: int,
                                n_docs: int, stream: int = 0) -> None:
        st = lib().ygm_merge_v1_device_lens_async(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_doc_off),
                                                  _dptr(d_upd_len), _dptr(d_doc_upd), n_upd, n_docs, stream or None)
        if st != OK:
            raise YjsError(st)

    def merge_device_finish(self) -> DeviceResult:
        """Completes the last enqueued batch (sequential tier, fault check, payload) -- ygm_merge_v1_device_finish."""
        r = _DevResult()
        st = lib().ygm_merge_v1_device_finish(self._ctx, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    def diff_device(self, d_arena, arena_bytes, d_doc_off, d_sv, d_sv_off, n_docs, stream=0) -> DeviceResult:
        r = _DevResult()
        st = lib().ygm_diff_v1_device(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_doc_off), _dptr(d_sv),
                                      _dptr(d_sv_off), n_docs, stream or None, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    def sv_device(self, d_arena, arena_bytes, d_doc_off, n_docs, stream=0) -> DeviceResult:
        r = _DevResult()
        st = lib().ygm_sv_from_update_v1_device(self._ctx, _dptr(d_arena, arena_bytes + TAIL_PAD), arena_bytes, _dptr(d_doc_off),
                                                n_docs, stream or None, ctypes.byref(r))
        if st != OK:
            raise YjsError(st)
        return DeviceResult(r.data, r.off, r.len, r.status, r.data_bytes, r.payload_bytes)

    def stats(self) -> Stats:
        s = Stats()
        lib().ygm_stats(self._ctx, ctypes.byref(s))
        return s
