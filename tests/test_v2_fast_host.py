"""The register-resident V1 -> V2 encoder (hocuspocus_amd/csrc/ygm_v2_fast.hpp, the k_v12_fast kernel's code)
host-compiled through tools/v2dev and compared byte for byte with the general transcoder (ygm_v2.hpp v12_body,
itself pinned by the yjs V2 vectors in tests/test_v2.py) on every V1 merge / diff output of the golden vectors and
on synthetic C2 merges.  Where the fast encoder takes a document it must produce the general path's bytes; where the
general path refuses or throws, the fast one must step aside."""
import ctypes
import os
import subprocess

import pytest

import oracle
from golden import load_yjs_vectors

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("v2dev") / "libv2dev.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "v2dev", "v2dev.cpp")],
                   check=True, timeout=600)
    L = ctypes.CDLL(so)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.hv_v12.argtypes = [vp, u32, vp, u64, u32, u32, vp, ctypes.POINTER(u64)]
    L.hv_v12f.argtypes = [vp, u32, vp, ctypes.POINTER(u64)]
    L.hv_v21.argtypes = [vp, u64, u32, u32, u32, vp, ctypes.POINTER(u64)]
    L.hv_v21f.argtypes = [vp, u32, u32, vp, ctypes.POINTER(u64)]
    return L


def general(L, v1):
    vb = ctypes.create_string_buffer(v1 + b"\0" * 64)
    ln = ctypes.c_uint64()
    e = L.hv_v12(vb, len(v1), vb, len(v1), 0, 0, None, ctypes.byref(ln))
    if e:
        return e, None
    out = ctypes.create_string_buffer(ln.value + 1)
    assert L.hv_v12(vb, len(v1), vb, len(v1), 0, 0, out, ctypes.byref(ln)) == 0
    return 0, out.raw[:ln.value]


def fast(L, v1):
    out = ctypes.create_string_buffer(8192)
    ln = ctypes.c_uint64()
    e = L.hv_v12f(v1, len(v1), out, ctypes.byref(ln))
    return e, out.raw[:ln.value] if e == 0 else None


def compare(L, v1s):
    took = 0
    for v1 in v1s:
        fe, fo = fast(L, v1)
        assert fe in (0, 1, 2), fe
        if fe == 0:
            ge, go = general(L, v1)
            assert (ge, go) == (0, fo), v1.hex()
            took += 1
    return took


def test_fast_v12_on_golden_outputs(lib):
    _, cases = load_yjs_vectors()
    v1s = []
    for c in cases:
        if c["out"] is not None and c["op"] in ("merge", "diff"):
            v1s.append(bytes.fromhex(c["out"]))
            if c["op"] == "merge":
                v1s.extend(bytes.fromhex(x) for x in c["in"])
    took = compare(lib, v1s)
    assert took > len(v1s) // 4, (took, len(v1s))


def test_fast_v12_on_c2_merges(lib):
    from tools import synth
    for seed, dp, run in ((5, 0, 1), (6, 20, 1), (7, 20, 16)):
        arena, upd_off, doc_upd = synth.text_updates(300, 60, seed=seed, del_pct=dp, max_run=run)
        ups = synth.split(arena, upd_off)
        v1s = [oracle.merge_updates(ups[doc_upd[d]:doc_upd[d + 1]])[1] for d in range(300)]
        assert compare(lib, v1s) == 300


def test_fast_v12_steps_aside(lib):
    # a non-ASCII string, a ContentType item, an empty block and a repeated client: the general path decides
    assert fast(lib, bytes.fromhex("0101050084010161c3a900"))[0] == 1   # string "aé" (UTF-8) -> not ASCII
    assert fast(lib, bytes.fromhex("010105000701016100"))[0] == 1       # ContentType
    assert fast(lib, bytes.fromhex("0200050001050000"))[0] == 1         # block of 0 structs


# ---------------------------------------------------------------- V2 -> V1 (ygm_v21_fast.hpp)
def general21(L, v2, mode):
    vb = ctypes.create_string_buffer(v2 + b"\0" * 64)
    ln = ctypes.c_uint64()
    e = L.hv_v21(vb, 0, len(v2), mode, 0, None, ctypes.byref(ln))
    if e:
        return e, None
    out = ctypes.create_string_buffer(ln.value + 1)
    assert L.hv_v21(vb, 0, len(v2), mode, 0, out, ctypes.byref(ln)) == 0
    return 0, out.raw[:ln.value]


def fast21(L, v2, mode):
    ln = ctypes.c_uint64()
    e = L.hv_v21f(v2, len(v2), mode, None, ctypes.byref(ln))
    if e:
        return e, None
    out = ctypes.create_string_buffer(ln.value + 1)
    assert L.hv_v21f(v2, len(v2), mode, out, ctypes.byref(ln)) == 0
    return 0, out.raw[:ln.value]


def compare21(L, v2s):
    took = 0
    for v2 in v2s:
        for mode in (0, 2):   # mergeUpdatesV2 / diffUpdateV2, encodeStateVectorFromUpdateV2 (structs only)
            fe, fo = fast21(L, v2, mode)
            assert fe in (0, 1), fe
            if fe == 0:
                assert general21(L, v2, mode) == (0, fo), (mode, v2.hex())
                took += 1
    return took


def test_fast_v21_on_golden_v2(lib):
    """Every V2 update of the yjs V2 vectors (merge / diff / sv inputs, outputs, conversion pairs, truncated and
    byte-flipped ones): where the fast transcoder takes it, the general transcoder's V1 bytes."""
    import gzip
    import json
    v2s = []
    with gzip.open(os.path.join(ROOT, "tests", "golden", "yjs13516_v2_vectors.jsonl.gz"), "rt") as f:
        next(f)
        for line in f:
            c = json.loads(line)
            keys = ("update",) if c["op"] == "sv_v2" else ("v2", "update", "out")   # (an sv_v2 output is a state vector)
            v2s.extend(bytes.fromhex(c[k]) for k in keys if isinstance(c.get(k), str))
            v2s.extend(bytes.fromhex(x) for x in c.get("in", []))
    took = compare21(lib, v2s)
    assert took > len(v2s) // 4, (took, len(v2s))


def test_fast_v21_on_c2_updates(lib):
    """C2 logs (single characters, 1-16-character runs, deletions, 1-8 clients) converted to V2 by the general
    encoder: every update is in the fast transcoder's shape."""
    from tools import synth
    for seed, dp, run, mx in ((5, 0, 1, 4), (6, 20, 1, 4), (7, 20, 16, 8)):
        arena, upd_off, _ = synth.text_updates(40, 50, 1, mx, seed=seed, del_pct=dp, max_run=run)
        v2s = []
        for v1 in synth.split(arena, upd_off):
            e, v2 = general(lib, v1)
            assert e == 0
            v2s.append(v2)
        assert compare21(lib, v2s) == 2 * len(v2s)
