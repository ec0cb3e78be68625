"""Compares snapshot outputs (tools/snapdev or the GPU) with the yjs expectations of tools/snap_corpus.js.
    python tools/snapdev/compare.py in.bin exp.bin got.bin"""
import collections
import struct
import sys


def read_in(f):
    b = open(f, "rb").read()
    n = struct.unpack_from("<I", b, 0)[0]
    i, out = 4, []
    for _ in range(n):
        ln = struct.unpack_from("<I", b, i)[0]
        i += 4
        out.append(b[i:i + ln])
        i += ln
    return out


def read_res(f):
    b = open(f, "rb").read()
    i, out = 0, []
    while i < len(b):
        st, ln = struct.unpack_from("<iI", b, i)
        i += 8
        out.append((st, b[i:i + ln]))
        i += ln
    return out


if __name__ == "__main__":
    ins, exp, got = read_in(sys.argv[1]), read_res(sys.argv[2]), read_res(sys.argv[3])
    c, bad = collections.Counter(), []
    for k, (e, g) in enumerate(zip(exp, got)):
        if g[0] != 0:
            c["status%d" % g[0]] += 1
        elif e[1] == g[1]:
            c["same"] += 1
        else:
            c["diff"] += 1
            bad.append(k)
    print(dict(c), "first diffs:", bad[:12])
    if bad and len(sys.argv) > 4:
        k = bad[int(sys.argv[4])]
        print("in ", ins[k].hex())
        print("exp", exp[k][1].hex())
        print("got", got[k][1].hex())
