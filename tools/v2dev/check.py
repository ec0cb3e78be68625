"""Development check of the device V2 transcoders on the CPU (host build, tools/v2dev/libv2dev.so): the V2
golden vectors through  v21 -> oracle V1 op -> v12  exactly as the GPU pipeline composes them.  Tooling only."""
import ctypes
import gzip
import json
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, "tools", "v2dev", "libv2dev.so"))
vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
L.hv_v21.argtypes = [vp, u64, u32, u32, u32, vp, ctypes.POINTER(u64)]
L.hv_v12.argtypes = [vp, u32, vp, u64, u32, u32, vp, ctypes.POINTER(u64)]
COMPAT = 1
THROW = {1, 2, 4, 5}


def v21(arena, off, n, mode):
    ab = (ctypes.c_uint8 * (len(arena) + 64)).from_buffer_copy(arena + b"\0" * 64)
    ln = u64()
    e = L.hv_v21(ab, off, n, mode, COMPAT, None, ctypes.byref(ln))
    if e:
        return e, None
    out = (ctypes.c_uint8 * (ln.value + 1))()
    e2 = L.hv_v21(ab, off, n, mode, COMPAT, out, ctypes.byref(ln))
    assert e2 == 0
    return 0, bytes(out[:ln.value])


def v12(v1, arena, mode):
    vb = (ctypes.c_uint8 * (len(v1) + 64)).from_buffer_copy(v1 + b"\0" * 64)
    ab = (ctypes.c_uint8 * (len(arena) + 64)).from_buffer_copy(arena + b"\0" * 64)
    ln = u64()
    e = L.hv_v12(vb, len(v1), ab, len(arena), mode, COMPAT, None, ctypes.byref(ln))
    if e:
        return e, None
    out = (ctypes.c_uint8 * (ln.value + 1))()
    e2 = L.hv_v12(vb, len(v1), ab, len(arena), mode, COMPAT, out, ctypes.byref(ln))
    assert e2 == 0, e2
    return 0, bytes(out[:ln.value])


def merge_v2(ups):
    if len(ups) == 1:
        return 0, ups[0]
    arena = b"".join(ups)
    offs = [0]
    for u in ups:
        offs.append(offs[-1] + len(u))
    v1s, err, ref = [], 0, 0
    for i, u in enumerate(ups):
        e, o = v21(arena, offs[i], len(u), 0)
        if e == 3:
            ref = ref or e
        elif e:
            err = err or e
        v1s.append(o or b"")
    if err or ref:
        return err or ref, None
    st, m = oracle.merge_updates(v1s, compat135=True)
    if st:
        return st, None
    return v12(m, arena, 0)


def diff_v2(u, sv):
    e, o = v21(u, 0, len(u), 0)
    if e:
        return e, None
    st, m = oracle.diff_update(o, sv, compat135=True)
    if st:
        return st, None
    return v12(m, u, 0)


def sv_v2(u):
    e, o = v21(u, 0, len(u), 2)
    if e:
        return e, None
    return oracle.encode_state_vector_from_update(o, compat135=True)


def main():
    lines = gzip.open(os.path.join(ROOT, "tests", "golden", "yjs13516_v2_vectors.jsonl.gz")).read().decode().splitlines()
    cases = [json.loads(x) for x in lines[1:]]
    bad = Counter()
    ex = {}
    for c in cases:
        op = c["op"]
        if op == "conv":
            v1, v2 = bytes.fromhex(c["v1"]), bytes.fromhex(c["v2"])
            r = v12(v1, b"", 1)
            if r != (0, v2):
                bad[("conv12", r[0])] += 1
                ex.setdefault(("conv12", r[0]), (c, r))
            r2 = v21(v2, 0, len(v2), 1)
            if not (r2[0] == 3 or r2 == (0, v1)):
                bad[("conv21", r2[0])] += 1
                ex.setdefault(("conv21", r2[0]), (c, r2))
            continue
        if op == "merge_v2":
            st, o = merge_v2([bytes.fromhex(x) for x in c["in"]])
        elif op == "diff_v2":
            st, o = diff_v2(bytes.fromhex(c["update"]), bytes.fromhex(c["sv"]))
        else:
            st, o = sv_v2(bytes.fromhex(c["update"]))
        exp = c["out"]
        b = c["family"].endswith("-bad")
        ok = (st in THROW or (st == 3 and b)) if exp is None else ((st == 0 and o.hex() == exp) or (st == 3 and b))
        if not ok:
            k = (op, b, st, exp is None)
            bad[k] += 1
            ex.setdefault(k, (c, (st, o and o.hex())))
    print("cases", len(cases), "bad", sum(bad.values()))
    for k, v in bad.items():
        print(v, k, json.dumps(ex[k][0])[:300], ex[k][1] if not isinstance(ex[k][1], tuple) else (ex[k][1][0], str(ex[k][1][1])[:200]))


if __name__ == "__main__":
    main()
