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


def ds_splice_docs(seed, n_docs=8):
    """[snapshot, ...log] documents over 16 KB whose snapshot delete set is large against the log's ranges (the
    large-document tier splices it instead of streaming it): log ranges before, inside, across, adjacent to and
    between the snapshot's ranges, zero-length ones, repeated ones, clients the snapshot has not got (before the
    first, between, after the last).  Documents 5.. also break the snapshot's delete set in ways the splice must
    refuse (adjacent or overlapping ranges, a zero-length range, an empty client, a non-minimal varuint): the
    union is then streamed, bit-exact either way."""
    rnd = random.Random(seed)
    docs = []
    for d in range(n_docs):
        nclients = rnd.choice([30, 200, 700])
        clients = sorted(rnd.sample(range(2, 1 << 28), nclients), reverse=True)
        # structs: one text block per client (the document is over 16 KB either way)
        snap = bytearray(_vu(len(clients)))
        for c in clients:
            txt = b"abcdefghij" * rnd.randint(2, 8) * (1 + 600 // nclients)
            snap += _vu(1) + _vu(c) + _vu(0) + bytes([0x04]) + _vu(1) + _vs(b"t") + _vs(txt)
        ds = {}
        for c in clients[:: rnd.choice([1, 2, 3])]:
            k, runs = rnd.randint(0, 50), []
            for _ in range(rnd.randint(1, 9000 // nclients)):
                ln = rnd.randint(1, 30)
                runs.append([k, ln])
                k += ln + rnd.randint(1, 40)
            ds[c] = runs
        broken = d >= 5
        if broken:
            c = rnd.choice(list(ds))
            r = ds[c]
            kind = d % 4
            if kind == 0 and len(r) > 1:
                r[1][0] = r[0][0] + r[0][1]                       # adjacent
            elif kind == 1 and len(r) > 1:
                r[1][0] = r[0][0] + r[0][1] - 1 if r[0][1] > 1 else r[0][0]   # overlapping
            elif kind == 2:
                r[-1][1] = 0                                      # zero-length
            else:
                ds[c] = []                                        # an empty client
        snap += _vu(len(ds))
        for c in sorted(ds, reverse=True):
            snap += _vu(c) + _vu(len(ds[c])) + b"".join(_vu(k) + _vu(ln) for k, ln in ds[c])
        if broken and d % 5 == 0:
            # a non-minimal varuint in the last range's length (0x81 0x00 = 1)
            assert snap[-1] < 0x80
            snap[-1:] = bytes([0x80 | snap[-1], 0x00])
        log = []
        dcl = sorted(ds)
        for _ in range(rnd.randint(3, 12)):
            rr = []
            for _ in range(rnd.randint(1, 10)):
                how = rnd.random()
                if how < 0.6 and dcl:
                    c = rnd.choice(dcl)
                    runs = ds[c] or [[5, 1]]
                    i = rnd.randrange(len(runs))
                    k0, ln0 = runs[i]
                    pick = rnd.randrange(8)
                    if pick == 0:
                        rr.append((c, k0 + ln0, rnd.randint(0, 3)))             # adjacent after
                    elif pick == 1:
                        rr.append((c, max(0, k0 - 2), 2))                       # adjacent / overlapping before
                    elif pick == 2:
                        rr.append((c, k0, ln0))                                 # the same range
                    elif pick == 3:
                        j = min(len(runs) - 1, i + rnd.randint(1, 5))
                        rr.append((c, k0 + 1, runs[j][0] + runs[j][1] - k0))   # across several
                    elif pick == 4:
                        rr.append((c, k0 + ln0 + 1, 0))                         # zero-length in a gap
                    elif pick == 5:
                        rr.append((c, runs[-1][0] + runs[-1][1] + rnd.randint(0, 9), rnd.randint(1, 4)))   # after the last
                    elif pick == 6:
                        rr.append((c, 0, rnd.randint(0, 3)))                    # at clock 0
                    else:
                        rr.append((c, k0 + ln0 // 2, 0))                        # zero-length inside
                else:
                    c = rnd.choice([1, clients[0] + rnd.randint(1, 9), rnd.randint(2, 1 << 28)])   # new clients
                    rr.append((c, rnd.randint(0, 100), rnd.randint(0, 5)))
            by = {}
            for c, k, ln in rr:
                by.setdefault(c, []).append((k, ln))
            u = bytearray(_vu(0) + _vu(len(by)))
            for c in sorted(by, reverse=True):   # a log update's own delete set: any order of ranges is fine
                u += _vu(c) + _vu(len(by[c])) + b"".join(_vu(k) + _vu(ln) for k, ln in by[c])
            log.append(bytes(u))
        docs.append([bytes(snap)] + log)
    return docs
