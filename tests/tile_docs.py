"""Hand-built [snapshot, ...log] V1 documents that probe the large-document kernel's LDS tiles (test data;
the GPU parity test and its CPU check import it)."""
import random


def _vu(n):
    out = bytearray()
    while n > 127:
        out.append(0x80 | (n & 127))
        n >>= 7
    out.append(n)
    return bytes(out)


def _vs(b):
    return _vu(len(b)) + b


def tile_edge_docs(seed, ds_ascending=False):
    """[snapshot, ...log] documents over 16 KB (the large-document tier) whose snapshots hold what the
    tiled walk must hand to global memory: strings longer than a tile's overlap (2 KB), ContentJSON
    with more entries than the speculative parse takes (64), structs straddling tile boundaries,
    more client blocks than one LDS staging refill (256), GC runs, a delete set; log updates touch
    clients between untouched (verbatim-run) blocks.  ds_ascending: the snapshot's delete set lists its
    clients in ascending order (not yjs's union order), which the large-document tier must hand on."""
    rnd = random.Random(seed)
    docs = []
    for d in range(6):
        nclients = [3, 40, 300, 600, 5, 1200][d]
        clients = sorted(rnd.sample(range(1, 1 << 30), nclients), reverse=True)
        blocks = []
        ends = {}
        for ci, c in enumerate(clients):
            structs = []
            clock = 0
            for q in range(rnd.randint(1, 4)):
                kind = rnd.random()
                if q == 0:
                    ln = 20000 if ci == 0 else rnd.choice([1, 5, 300, 2100, 5000]) if kind < 0.3 else rnd.randint(1, 40)
                    txt = "".join(rnd.choice("abcdefgh ") for _ in range(ln)).encode()
                    structs.append(bytes([0x04]) + _vu(1) + _vs(b"t") + _vs(txt))
                    clock += ln
                elif kind < 0.2:
                    structs.append(bytes([0x00]) + _vu(7))                       # GC
                    clock += 7
                elif kind < 0.35:
                    n = rnd.choice([3, 65, 100])                               # ContentJSON
                    structs.append(bytes([0x82]) + _vu(c) + _vu(clock - 1) + _vu(n) + b"".join(_vs(b"1") for _ in range(n)))
                    clock += n
                else:
                    ln = rnd.choice([1, 3, 2500])
                    txt = "".join(rnd.choice("xyz") for _ in range(ln)).encode()
                    structs.append(bytes([0x84]) + _vu(c) + _vu(clock - 1) + _vs(txt))
                    clock += ln
            # GC structs never follow each other (yjs merges them)
            fixed = [structs[0]]
            for st in structs[1:]:
                if st[0] == 0 and fixed[-1][0] == 0:
                    continue
                fixed.append(st)
            blocks.append((c, fixed))
        snap = bytearray(_vu(len(blocks)))
        for c, structs in blocks:
            snap += _vu(len(structs)) + _vu(c) + _vu(0) + b"".join(structs)
        dcl = clients[: max(2, nclients // 10)]
        if ds_ascending:
            dcl = dcl[::-1]
        snap += _vu(len(dcl))
        for c in dcl:
            snap += _vu(c) + _vu(1) + _vu(0) + _vu(1)
        log = []
        for c in rnd.sample(clients, min(len(clients), 8)):
            log.append(_vu(1) + _vu(1) + _vu(c) + _vu(1 << 20) + bytes([0x04]) + _vu(1) + _vs(b"t") + _vs(b"q") + _vu(0))
        log.append(_vu(0) + _vu(1) + _vu(clients[-1]) + _vu(1) + _vu(2) + _vu(3))    # a deletion
        docs.append([bytes(snap)] + log)
    return docs
