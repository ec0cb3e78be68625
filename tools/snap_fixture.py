"""Builds a snapshot fixture file for tests/golden (tooling): runs tools/snap_corpus.js (the image's yjs 13.5.16 bundle)
once per (n, seed, maxOps, mode) part and writes {"source": ..., "rows": [[update hex, expected hex], ...]} gzipped.

    python tools/snap_fixture.py OUT.json.gz N:SEED:MAXOPS:MODE [...]
    python tools/snap_fixture.py --contains OUT.json.gz N SEED [pending]    (tools/contains_corpus.js: states, rows)

tests/golden/snapshot_pending_v135.json.gz: 200:31:120:pending 120:32:200:textpending
tests/golden/contains_pending_v135.json.gz: --contains 120 51 pending"""
import gzip
import json
import os
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read_in(path):
    b = open(path, "rb").read()
    n, i, out = struct.unpack_from("<I", b, 0)[0], 4, []
    for _ in range(n):
        ln = struct.unpack_from("<I", b, i)[0]
        out.append(b[i + 4:i + 4 + ln])
        i += 4 + ln
    return out


def _read_exp(path):
    b = open(path, "rb").read()
    i, out = 0, []
    while i < len(b):
        st, ln = struct.unpack_from("<iI", b, i)
        out.append(b[i + 8:i + 8 + ln])
        i += 8 + ln
    return out


def contains(out, n, seed, mode):
    with tempfile.TemporaryDirectory() as t:
        a, b, c = (os.path.join(t, x) for x in ("s.bin", "u.bin", "e.bin"))
        subprocess.run(["node", os.path.join(ROOT, "tools", "contains_corpus.js"), n, seed, a, b, c] + ([mode] if mode else []), check=True)
        states, updates, exp = _read_in(a), _read_in(b), open(c, "rb").read()
    uniq, idx = [], {}
    for st in states:
        if st not in idx:
            idx[st] = len(uniq)
            uniq.append(st)
    rows = [[idx[st], u.hex(), int(e)] for st, u, e in zip(states, updates, exp)]
    src = f"node tools/contains_corpus.js {n} {seed} {mode} (yjs 13.5.16 bundle) via tools/snap_fixture.py --contains"
    with gzip.open(out, "wt") as f:
        json.dump({"source": src, "states": [x.hex() for x in uniq], "rows": rows}, f)
    print(len(rows), "rows", len(uniq), "states")


def main():
    if sys.argv[1] == "--contains":
        return contains(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else "")
    out, parts = sys.argv[1], sys.argv[2:]
    rows = []
    with tempfile.TemporaryDirectory() as t:
        for p in parts:
            n, seed, ops, mode = p.split(":")
            a, b = os.path.join(t, "in.bin"), os.path.join(t, "exp.bin")
            subprocess.run(["node", os.path.join(ROOT, "tools", "snap_corpus.js"), n, seed, a, b, ops, mode], check=True)
            rows += [[u.hex(), e.hex()] for u, e in zip(_read_in(a), _read_exp(b))]
    src = "tools/snap_corpus.js (yjs 13.5.16 bundle) via tools/snap_fixture.py " + " ".join(parts)
    with gzip.open(out, "wt") as f:
        json.dump({"source": src, "rows": rows}, f)
    print(len(rows), "rows")


if __name__ == "__main__":
    main()
