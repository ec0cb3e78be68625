"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle and the
yjs golden vectors.  One process, batched calls (each call = one kernel batch)."""
import random

import numpy as np
import pytest

import oracle
from golden import case_inputs, check_result, load_yjs_vectors
from hocuspocus_amd.engine import EMALFORMED

pytestmark = pytest.mark.gpu

HEADER, CASES = load_yjs_vectors()
THROWS = {1, 2, 4, 5}


@pytest.fixture(scope="module")
def eng():
    from hocuspocus_amd import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng135():
    from hocuspocus_amd import Engine
    e = Engine(0, compat135=True)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng_seq():
    from hocuspocus_amd import Engine
    e = Engine(0, force_seq=True)
    yield e
    e.close()


def same(oracle_res, gpu_res):
    """statuses agree (any throw == any throw) and bytes agree when OK."""
    so, bo = oracle_res
    sg, bg = gpu_res
    if so in THROWS:
        return sg in THROWS
    return so == sg and bo == bg


def run_batch(e, op, cases):
    if op == "merge":
        return e.merge_updates_batch([case_inputs(c) for c in cases])
    if op == "diff":
        ins = [case_inputs(c) for c in cases]
        return e.diff_update_batch([u for u, _ in ins], [s for _, s in ins])
    return e.encode_state_vector_from_update_batch([case_inputs(c) for c in cases])


@pytest.mark.parametrize("op", ["merge", "diff", "sv"])
def test_golden_vectors_compat135(eng135, op):
    cases = [c for c in CASES if c["op"] == op]
    res = run_batch(eng135, op, cases)
    bad = []
    for c, (st, out) in zip(cases, res):
        why = check_result(c, st, out)
        if why:
            bad.append((c["id"], c.get("note"), why))
    assert not bad, f"{len(bad)} of {len(cases)} differ; first {bad[:3]}"


@pytest.mark.parametrize("op", ["merge", "diff", "sv"])
def test_golden_inputs_default_mode_vs_oracle(eng, op):
    cases = [c for c in CASES if c["op"] == op]
    res = run_batch(eng, op, cases)
    bad = []
    for c, g in zip(cases, res):
        if op == "merge":
            o = oracle.merge_updates(case_inputs(c))
        elif op == "diff":
            o = oracle.diff_update(*case_inputs(c))
        else:
            o = oracle.encode_state_vector_from_update(case_inputs(c))
        if not same(o, g):
            bad.append((c["id"], c.get("note"), o[0], g[0]))
    assert not bad, f"{len(bad)} of {len(cases)} differ; first {bad[:5]}"


def test_sequential_kernel_on_golden_merges(eng_seq):
    cases = [c for c in CASES if c["op"] == "merge"]
    res = run_batch(eng_seq, "merge", cases)
    bad = []
    for c, g in zip(cases, res):
        o = oracle.merge_updates(case_inputs(c))
        if not same(o, g):
            bad.append((c["id"], c.get("note"), o[0], g[0]))
    assert not bad, f"{len(bad)} of {len(cases)} differ; first {bad[:5]}"


def _synth_docs(n_docs, n_upd, seed, del_pct=0, shuffle=False):
    from tools import synth
    arena, upd_off, doc_upd = synth.text_updates(n_docs, n_upd, seed=seed, del_pct=del_pct)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(n_docs)]
    if shuffle:
        rng = random.Random(seed)
        for d in docs:
            rng.shuffle(d)
    return docs


@pytest.mark.parametrize("del_pct,shuffle", [(0, False), (20, False), (20, True)])
def test_synthetic_c2_merge_vs_oracle(eng, del_pct, shuffle):
    docs = _synth_docs(600, 200, seed=5 + del_pct, del_pct=del_pct, shuffle=shuffle)
    seq0 = eng.stats().docs_seq
    res = eng.merge_updates_batch(docs)
    for d, us in enumerate(docs):
        assert same(oracle.merge_updates(us), res[d]), d
    # yjs-produced (sorted, overlap-free) updates never need the sequential kernel
    assert eng.stats().docs_seq == seq0


def test_merge_with_duplicates_and_premerged(eng):
    # overlap class: duplicated updates and overlapping pre-merged halves -> sequential kernel
    rng = random.Random(9)
    docs = _synth_docs(200, 60, seed=9, del_pct=10)
    batch = []
    for us in docs:
        x = list(us)
        x += rng.sample(us, 3)
        rng.shuffle(x)
        a = oracle.merge_updates(us[:40])[1]
        b = oracle.merge_updates(us[20:])[1]
        batch += [x, [a, b], [b, a] + us[:5]]
    res = eng.merge_updates_batch(batch)
    for i, us in enumerate(batch):
        assert same(oracle.merge_updates(us), res[i]), i


def test_synthetic_c4_sv_and_diff_vs_oracle(eng):
    from tools import synth
    arena, doc_off, sva, sv_off = synth.text_states(800, seed=21)
    docs = synth.split(arena, doc_off)
    svs = synth.split(sva, sv_off)
    res = eng.encode_state_vector_from_update_batch(docs)
    for d, u in enumerate(docs):
        assert same(oracle.encode_state_vector_from_update(u), res[d]), d
    res = eng.diff_update_batch(docs, svs)
    for d, u in enumerate(docs):
        assert same(oracle.diff_update(u, svs[d]), res[d]), d


def test_fuzzed_inputs_vs_oracle(eng):
    # truncations and byte flips of real inputs: error class and bytes must agree
    rng = random.Random(1234)
    merges, diffs, svs = [], [], []
    pool = [c for c in CASES if c["out"] is not None]
    for _ in range(3000):
        c = rng.choice(pool)
        if c["op"] == "merge":
            us = [bytearray(u) for u in case_inputs(c)]
            if len(us) < 2:
                continue
            u = rng.choice(us)
            if u and rng.random() < 0.5:
                u[rng.randrange(len(u))] = rng.randrange(256)
            elif u:
                del u[rng.randrange(len(u)):]
            merges.append([bytes(x) for x in us])
        elif c["op"] == "diff":
            u, s = case_inputs(c)
            u = bytearray(u)
            if u:
                u[rng.randrange(len(u))] ^= 1 << rng.randrange(8)
            diffs.append((bytes(u), s))
        else:
            u = bytearray(case_inputs(c))
            if u:
                del u[rng.randrange(len(u)):]
            svs.append(bytes(u))
    res = eng.merge_updates_batch(merges)
    for us, g in zip(merges, res):
        assert same(oracle.merge_updates(us), g), [u.hex() for u in us]
    res = eng.diff_update_batch([u for u, _ in diffs], [s for _, s in diffs])
    for (u, s), g in zip(diffs, res):
        assert same(oracle.diff_update(u, s), g), (u.hex(), s.hex())
    res = eng.encode_state_vector_from_update_batch(svs)
    for u, g in zip(svs, res):
        assert same(oracle.encode_state_vector_from_update(u), g), u.hex()


def test_empty_and_edge_batches(eng):
    assert eng.merge_updates_batch([]) == []
    assert eng.merge_updates_batch([[]]) == [(0, bytes.fromhex("0000"))]
    one = bytes.fromhex("01010500040101740568656c6c6f00")
    assert eng.merge_updates_batch([[one]]) == [(0, one)]
    assert eng.merge_updates_batch([[b"\x01"]]) == [(0, b"\x01")]  # single input: returned as-is
    r = eng.merge_updates_batch([[b"\x01", b"\x00\x00"], [one, one]])
    assert r[0][0] in THROWS and r[1] == (0, one)


def test_full_size_c2_properties(eng):
    # BASELINE configs[1] size (10k docs x 200 updates): size-independent properties
    from tools import synth
    arena, upd_off, doc_upd = synth.text_updates(10000, 200, seed=1)
    res = eng.merge_packed(arena, upd_off, doc_upd[:-1].repeat(np.diff(doc_upd)) if False else
                           np.repeat(np.arange(10000, dtype=np.uint32), np.diff(doc_upd).astype(np.int64)), 10000)
    assert all(st == 0 for st, _ in res)
    merged = [m for _, m in res]
    # (1) diff against an empty state vector reproduces a canonical merged update
    d = eng.diff_update_batch(merged, [b"\x00"] * len(merged))
    assert all(x == (0, m) for x, m in zip(d, merged))
    # (2) every insert is present: SV clocks sum to the number of updates
    svs = eng.encode_state_vector_from_update_batch(merged)
    from v1util import rd_vu
    for st, sv in svs[:2000]:
        n, p = rd_vu(sv, 0)
        tot = 0
        for _ in range(n):
            _, p = rd_vu(sv, p)
            k, p = rd_vu(sv, p)
            tot += k
        assert tot == 200
    # (3) spot-check against the oracle
    ups = synth.split(arena, upd_off)
    for dd in range(0, 10000, 97):
        assert (0, merged[dd]) == oracle.merge_updates(ups[doc_upd[dd]:doc_upd[dd + 1]])


def test_lean_kernel_takes_debounce_logs(eng):
    # C2-shaped logs (1-8 clients, per-client clock order, with or without deletions) are
    # finished by the lean kernel; 9+ clients and shuffled logs are deferred -- all bit-exact.
    from tools import synth
    cases = [(dict(min_clients=1, max_clients=4), 0, False, True),
             (dict(min_clients=5, max_clients=8), 0, False, True),
             (dict(min_clients=9, max_clients=12), 0, False, False),
             (dict(min_clients=6, max_clients=8), 20, False, True),
             (dict(min_clients=1, max_clients=4), 0, True, None),
             (dict(min_clients=1, max_clients=3), 15, False, True),
             (dict(min_clients=1, max_clients=4), 20, False, True)]
    for kw, del_pct, shuffle, all_lean in cases:
        arena, upd_off, doc_upd = synth.text_updates(300, 120, del_pct=del_pct, seed=77, **kw)
        ups = synth.split(arena, upd_off)
        docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(300)]
        if shuffle:
            rng = random.Random(3)
            for dd in docs:
                rng.shuffle(dd)
        lean0 = eng.stats().docs_lean
        res = eng.merge_updates_batch(docs)
        for d, us in enumerate(docs):
            assert same(oracle.merge_updates(us), res[d]), (kw, del_pct, shuffle, d)
        took = eng.stats().docs_lean - lean0
        if all_lean is True:
            assert took == 300
        elif all_lean is False:
            assert took == 0


def test_wide_lean_kernel_takes_mixed_logs(eng):
    # c2_mixed shape (bench.py mixed_block): 1-8 clients, 1-16 character inserts (updates of up to ~42
    # bytes), 20 % deletions -- past the narrow kernel's 32-byte window, finished by the wide lean kernel
    from tools import synth
    n = 2000
    arena, upd_off, doc_upd = synth.text_updates(n, 200, 1, 8, del_pct=20, seed=71, max_run=16)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(n)]
    s0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), bad[:5])
    s1 = eng.stats()
    assert s1.docs_lean - s0.docs_lean >= 0.9 * n
    assert s1.docs_lean_wide - s0.docs_lean_wide >= 0.9 * n


def test_wide_route_with_deferrals_and_passthrough(eng):
    # a batch whose average document is past the narrow kernel's staging takes the wide kernel over every document
    # (the wide route): documents it defers (duplicated updates: overlaps for the general tiers), single-update and
    # empty documents (passed through) must come out as they do through the narrow route
    from tools import synth
    rng = random.Random(9)
    arena, upd_off, doc_upd = synth.text_updates(1500, 200, 1, 8, del_pct=20, seed=72, max_run=16)
    ups = synth.split(arena, upd_off)
    mixed = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(1500)]
    docs = []
    for i in range(3000):
        r = rng.random()
        m = mixed[i % 1500]
        docs.append([] if r < 0.04 else [m[0]] if r < 0.12 else m + m[: len(m) // 3] if r < 0.3 else m)
    assert sum(len(u) for us in docs for u in us) / len(docs) > 5120   # (the wide route's condition)
    s0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), bad[:5])
    s1 = eng.stats()
    assert s1.docs_lean_wide - s0.docs_lean_wide > 0 and (s1.docs - s0.docs) - (s1.docs_lean - s0.docs_lean) > 0   # (some deferred)


def test_lean_deferrals_beside_single_update_documents(eng):
    # more documents than the narrow kernel's persistent grid, so every wave takes several: single-update
    # and empty documents (passed through, not parsed) between documents the narrow kernel defers must not
    # shift the wave's record of which documents it deferred
    from tools import synth
    rng = random.Random(5)
    arena, upd_off, doc_upd = synth.text_updates(3000, 30, 9, 12, seed=13)         # 9+ clients: deferred
    ups = synth.split(arena, upd_off)
    deferred = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(3000)]
    arena, upd_off, doc_upd = synth.text_updates(3000, 30, 1, 3, seed=14)          # lean
    ups = synth.split(arena, upd_off)
    lean = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(3000)]
    docs = []
    for i in range(12000):
        r = rng.random()
        docs.append([] if r < 0.1 else [lean[i % 3000][0]] if r < 0.4 else deferred[i % 3000] if r < 0.6 else lean[i % 3000])
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), bad[:5])


def _lean_edge_docs(n_docs, seed):
    """Debounce-log-like documents whose updates probe every branch of the lean kernel's
    parser: string lengths around the 32-byte window, non-ASCII, ContentDeleted, parent
    keys / ids, parentSub with and without origins, non-minimal varuints, 5-byte clients
    (some >= 2^32), large clocks, multi-struct updates, trailing bytes, gaps and overlaps."""
    from v1util import vu
    rng = random.Random(seed)
    docs = []
    for _ in range(n_docs):
        ncl = rng.choice([1, 1, 2, 3, 4, 5])
        clients = [rng.choice([rng.randrange(1, 2 ** 32), rng.randrange(1, 200), 2 ** 32 + rng.randrange(5)])
                   if rng.random() < 0.1 else rng.randrange(1, 2 ** 32) for _ in range(ncl)]
        clocks = [rng.choice([0, 0, 0, rng.randrange(2 ** 28, 2 ** 31)]) for _ in range(ncl)]
        ups = []
        for _ in range(rng.randrange(2, 60)):
            c = rng.randrange(ncl)
            nst = 1 if rng.random() < 0.85 else rng.randrange(2, 4)
            body = bytearray()
            clen_total = 0
            for _s in range(nst):
                kind = rng.random()
                nm = rng.random() < 0.03
                def id_(cl, ck):
                    b = vu(cl) + vu(ck)
                    return b[:-1] + bytes([b[-1] | 0x80, 0]) if nm else b
                info, extra = 0, b""
                shape = rng.random()
                if shape < 0.6:
                    info |= 0x80 | 0x40
                    extra = id_(rng.choice(clients), rng.randrange(300)) + id_(rng.choice(clients), rng.randrange(300))
                elif shape < 0.7:
                    info |= 0x80
                    extra = id_(rng.choice(clients), rng.randrange(300))
                elif shape < 0.8:
                    info |= 0x40
                    extra = id_(rng.choice(clients), rng.randrange(300))
                elif shape < 0.9:
                    extra = b"\x01" + vu(1) + b"t"                    # parent ykey
                    if rng.random() < 0.5:
                        info |= 0x20
                        extra += vu(3) + b"key"                      # parentSub
                else:
                    extra = b"\x00" + id_(rng.choice(clients), rng.randrange(50))   # parent id
                if shape < 0.8 and rng.random() < 0.05:
                    info |= 0x20                                     # dropped on re-encode (origin present)
                if kind < 0.8:
                    ln = rng.choice([1, 1, 1, 2, 5, 20, 31, 32, 40])
                    txt = "".join(rng.choice("abcdefgh") for _ in range(ln))
                    if rng.random() < 0.05:
                        txt = txt[:-1] + "é"
                    raw = txt.encode()
                    info |= 4
                    content = vu(len(raw)) + raw
                    clen = len(txt.encode("utf-16-le")) // 2
                else:
                    clen = rng.choice([1, 3, 200, 70000])
                    info |= 1
                    content = vu(clen)
                body += bytes([info]) + extra + content
                clen_total += clen
            ck = clocks[c]
            if rng.random() < 0.02:
                ck += 1                                              # gap
            elif rng.random() < 0.02 and ck > 0:
                ck -= 1                                              # overlap
            u = vu(1) + vu(nst) + vu(clients[c]) + vu(ck) + bytes(body) + b"\x00"
            if rng.random() < 0.02:
                u += b"\x07\x07"                                     # trailing bytes: ignored by yjs
            ups.append(u)
            clocks[c] = ck + clen_total
        docs.append(ups)
    return docs


def test_lean_kernel_edge_shapes_vs_oracle(eng):
    docs = _lean_edge_docs(1500, seed=4242)
    lean0 = eng.stats().docs_lean
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), [u.hex() for u in docs[bad[0]]])
    took = eng.stats().docs_lean - lean0
    assert 0 < took < len(docs)   # both the lean path and the deferral path are exercised


def test_async_device_api_matches_host_api(eng):
    # ygm_merge_v1_device_async + finish (what bench.py times) == the host API, including a batch
    # whose documents need every tier (lean, wave, workgroup, sequential)
    import torch
    from tools import synth
    from v1util import vu  # noqa: F401
    arena, upd_off, doc_upd = synth.text_updates(400, 120, seed=31, del_pct=10)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(400)]
    rng = random.Random(5)
    for d in range(0, 400, 7):
        docs[d] = docs[d] + rng.sample(docs[d], 2)          # duplicates: the sequential tier
    docs += _lean_edge_docs(100, seed=77)
    blobs = [u for us in docs for u in us]
    a = np.frombuffer(b"".join(blobs) + bytes(64), np.uint8)
    off = np.cumsum([0] + [len(b) for b in blobs]).astype(np.uint64)
    du = np.cumsum([0] + [len(us) for us in docs]).astype(np.uint32)
    dev = torch.device("cuda", 0)
    ta, to, td = (torch.from_numpy(x.copy()).to(dev) for x in (a, off.view(np.int64), du.view(np.int32)))
    for _ in range(2):   # the second enqueue reuses the context's buffers
        eng.merge_device_async(ta.data_ptr(), len(a) - 64, to.data_ptr(), td.data_ptr(), len(blobs), len(docs))
    r = eng.merge_device_finish()
    torch.cuda.synchronize()
    import bench
    n = len(docs)
    offs = bench._d2h(r.off, n * 8).view(np.uint64)
    lens = bench._d2h(r.len, n * 8).view(np.uint64)
    sts = bench._d2h(r.status, n * 4).view(np.int32)
    data = bench._d2h(r.data, int(r.data_bytes)).tobytes()
    host = eng.merge_updates_batch(docs)
    for d in range(n):
        got = (int(sts[d]), data[int(offs[d]):int(offs[d]) + int(lens[d])] if sts[d] == 0 else None)
        assert got[0] == host[d][0] and (got[0] != 0 or got[1] == host[d][1]), d
    assert r.payload_bytes == sum(len(h[1]) for h in host if h[0] == 0)


def _lens_check(eng, docs, bad_lens):
    # docs through ygm_merge_v1_device_lens with the lengths bad_lens {update index: length} changed: the documents
    # holding a changed update get YGM_EMALFORMED on every route (the single-update check, the lean kernels, the
    # empty updates k_build_off leaves to the general tiers), every other one the host API's result
    import torch
    import bench
    blobs = [u for us in docs for u in us]
    assert max(len(b) for b in blobs) < 65536
    a = np.frombuffer(b"".join(blobs) + bytes(64), np.uint8)
    lens = np.array([len(b) for b in blobs], np.uint16)
    du = np.cumsum([0] + [len(us) for us in docs]).astype(np.uint32)
    doff = np.cumsum([0] + [sum(len(u) for u in us) for us in docs]).astype(np.uint64)
    for u, v in bad_lens.items():
        lens[u] = v
    bad = {int(np.searchsorted(du, u, side="right")) - 1 for u in bad_lens}
    dev = torch.device("cuda", 0)
    ta, to, tl, td = (torch.from_numpy(x.copy()).to(dev) for x in (a, doff.view(np.int64), lens.view(np.int16), du.view(np.int32)))
    n = len(docs)
    host = eng.merge_updates_batch(docs)
    for _ in range(2):   # the second call reuses the context's buffers
        r = eng.merge_device_lens(ta.data_ptr(), len(a) - 64, to.data_ptr(), tl.data_ptr(), td.data_ptr(), len(blobs), n)
        torch.cuda.synchronize()
        offs = bench._d2h(r.off, n * 8).view(np.uint64)
        ln = bench._d2h(r.len, n * 8).view(np.uint64)
        sts = bench._d2h(r.status, n * 4).view(np.int32)
        data = bench._d2h(r.data, int(r.data_bytes)).tobytes()
        for d in range(n):
            got = (int(sts[d]), data[int(offs[d]):int(offs[d]) + int(ln[d])] if sts[d] == 0 else None)
            if d in bad:
                assert got[0] == EMALFORMED, (d, got[0])
            else:
                assert got[0] == host[d][0] and (got[0] != 0 or got[1] == host[d][1]), d


def _device_merge(eng, docs):
    # docs through ygm_merge_v1_device: (status, bytes) per document, and the call's host waits (ygm_stats host_syncs)
    import torch
    import bench
    blobs = [u for us in docs for u in us]
    a = np.frombuffer(b"".join(blobs) + bytes(64), np.uint8)
    off = np.cumsum([0] + [len(b) for b in blobs]).astype(np.uint64)
    du = np.cumsum([0] + [len(us) for us in docs]).astype(np.uint32)
    dev = torch.device("cuda", 0)
    ta, to, td = (torch.from_numpy(x.copy()).to(dev) for x in (a, off.view(np.int64), du.view(np.int32)))
    s0 = eng.stats()
    r = eng.merge_device(ta.data_ptr(), len(a) - 64, to.data_ptr(), td.data_ptr(), len(blobs), len(docs))
    s1 = eng.stats()
    syncs = {"syncs": s1.host_syncs - s0.host_syncs, "general": (s1.docs_fast - s0.docs_fast) + (s1.docs_big - s0.docs_big),
             "large_or_seq": (s1.docs_big - s0.docs_big) + (s1.docs_seq - s0.docs_seq)}
    torch.cuda.synchronize()
    n = len(docs)
    offs = bench._d2h(r.off, n * 8).view(np.uint64)
    lens = bench._d2h(r.len, n * 8).view(np.uint64)
    sts = bench._d2h(r.status, n * 4).view(np.int32)
    data = bench._d2h(r.data, int(r.data_bytes)).tobytes()
    return [(int(sts[d]), data[int(offs[d]):int(offs[d]) + int(lens[d])] if sts[d] == 0 else None) for d in range(n)], syncs


def test_host_syncs_per_merge_call(eng):
    # the general tiers run chained on the device (wide -> wave -> workgroup, each reading its count from
    # the counters the kernel before it wrote), so a call waits on the device once for a batch the lean kernels finish,
    # twice for one that needs the general tiers, and more only for large documents (their scratch is sized from the
    # counters) -- every result still the oracle's
    from tools import synth
    a, o, dd = synth.text_updates(300, 200, seed=81)
    ups = synth.split(a, o)
    c2 = [ups[dd[d]:dd[d + 1]] for d in range(300)]
    a, o, dd = synth.text_updates(40, 200, 9, 16, del_pct=10, seed=82)   # 9-16 clients: past the lean kernels' 8 -> the wave tier
    ups = synth.split(a, o)
    wave = c2[:200] + [ups[dd[d]:dd[d + 1]] for d in range(40)]
    a, o, dd = synth.text_updates(20, 250, 9, 16, seed=84, max_run=30)   # ~10 KB: past the wave tier's 8 KB -> the workgroup tier
    ups = synth.split(a, o)
    fast = c2[:200] + [ups[dd[d]:dd[d + 1]] for d in range(20)]
    rng = random.Random(9)
    a, o, dd = synth.big_docs(3, 200000, 64 * 1024, max_clients=64, max_k=50, seed=83)
    ups = synth.split(a, o)
    big = c2[:100] + [ups[dd[d]:dd[d + 1]] for d in range(3)]
    rng.shuffle(big)
    general_only = 0
    seen = []
    for docs in (c2, wave, fast, big):
        res, k = _device_merge(eng, docs)
        seen.append(k)
        bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
        assert not bad, (len(bad), bad[:5])
        if docs is c2:
            assert k["syncs"] == 1 and k["general"] == 0, k
        elif k["large_or_seq"] == 0:   # the general tiers only: one wait for all of them
            assert k["syncs"] == 2, k
            general_only += k["general"] > 0
        else:   # + the large-document tier (scratch sizing, the scan's lists, the mid size's deferrals) / sequential
            assert k["syncs"] <= 6, k
    assert general_only >= 1, seen


def test_compact_lens_device_api_matches_host_api(eng):
    # ygm_merge_v1_device_lens (u64 per document, u16 length per update) == the host API on a batch that needs every
    # tier (the deferred documents' offsets are built on the device); documents whose lengths do not add up to their
    # bytes get an error status: lengths past the bytes, short of them (two or more updates), a single update's
    # length other than the document's bytes
    from tools import synth
    arena, upd_off, doc_upd = synth.text_updates(400, 120, seed=32, del_pct=10)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(400)]
    rng = random.Random(6)
    for d in range(0, 400, 7):
        docs[d] = docs[d] + rng.sample(docs[d], 2)          # duplicates: the sequential tier
    docs += _lean_edge_docs(100, seed=78)
    ba, bo, bd = synth.big_docs(3, 60000, 1024, max_clients=16, max_k=40, seed=7)   # the large-document tier
    bu = synth.split(ba, bo)
    docs += [bu[bd[d]:bd[d + 1]] for d in range(3)]
    docs += [[ups[3]], [ups[4]]]                                  # single-update documents (passed through)
    du = np.cumsum([0] + [len(us) for us in docs]).astype(np.uint32)
    lens = [len(u) for us in docs for u in us]
    _lens_check(eng, docs, {int(du[5]): lens[du[5]] + 3,           # past the bytes
                            int(du[12]) + 1: lens[du[12] + 1] - 1,  # short of them
                            int(du[401]): lens[du[401]] - 1,        # an edge document (wave / workgroup tiers)
                            int(du[len(docs) - 1]): lens[du[len(docs) - 1]] + 1})   # a single update
    # the wide route (the batch's average document outgrows the narrow kernel's staging: every document takes the
    # wide kernel, the table built whole on the device)
    wa, wo, wd = synth.text_updates(300, 200, 1, 8, del_pct=20, seed=71, max_run=16)
    wu = synth.split(wa, wo)
    wdocs = [wu[wd[d]:wd[d + 1]] for d in range(300)] + [[wu[7]], [wu[9]]]
    wdu = np.cumsum([0] + [len(us) for us in wdocs]).astype(np.uint32)
    wl = [len(u) for us in wdocs for u in us]
    _lens_check(eng, wdocs, {int(wdu[3]) + 2: wl[wdu[3] + 2] - 2, int(wdu[301]): wl[wdu[301]] + 2})


def test_lean_sv_diff_edge_states_vs_oracle(eng):
    # merged states with every struct shape of the lean-edge corpus (long strings, non-ASCII, deleted
    # content, parents, 5-byte clients, large clocks, multi-struct blocks), diffed against random state
    # vectors (missing clients, clocks inside / at / past each client's range, repeated entries)
    from v1util import vu
    rng = random.Random(99)
    states, svs = [], []
    for us in _lean_edge_docs(600, seed=2024):
        st, m = oracle.merge_updates(us)
        if st != 0:
            continue
        states.append(m)
        svst, sv = oracle.encode_state_vector_from_update(m)
        ents = []
        if svst == 0 and sv:
            n, p = 0, 0
            from v1util import rd_vu
            n, p = rd_vu(sv, 0)
            for _ in range(n):
                c, p = rd_vu(sv, p)
                k, p = rd_vu(sv, p)
                ents.append((c, rng.choice([0, k, max(k - 1, 0), rng.randrange(k + 1), k + 5])))
        rng.shuffle(ents)
        if ents and rng.random() < 0.2:
            ents.append(ents[0])                       # repeated client: the last entry wins
        if rng.random() < 0.1:
            ents = []
        svs.append(vu(len(ents)) + b"".join(vu(c) + vu(k) for c, k in ents))
    lean0 = eng.stats().docs_lean
    res = eng.encode_state_vector_from_update_batch(states)
    for d, u in enumerate(states):
        assert same(oracle.encode_state_vector_from_update(u), res[d]), u.hex()
    res = eng.diff_update_batch(states, svs)
    for d, u in enumerate(states):
        assert same(oracle.diff_update(u, svs[d]), res[d]), (u.hex(), svs[d].hex())
    took = eng.stats().docs_lean - lean0
    assert 0 < took < 2 * len(states)


def _walker_states(n_docs, seed):
    """Merged-state-shaped updates for the SV / diff ring walker: 0-20 client blocks (mostly strictly
    descending, 5-byte and small clients, first clocks 0 or large), strings of 1-300 bytes (past the
    64-byte mask window and the 256-byte ring), non-ASCII strings, ContentDeleted, GC (canonical and
    not), Skips, ContentType with keys, ContentBinary, parent ids / y-keys / parentSub, delete sets
    (descending or not, empty clients), truncations and trailing bytes."""
    from v1util import vu
    rng = random.Random(seed)
    docs, ends = [], []
    for _ in range(n_docs):
        nb = rng.choice([0, 1, 1, 2, 3, 5, 8, 12, 16, 20])
        cl = set()
        while len(cl) < nb:
            cl.add(rng.choice([rng.randrange(1, 2 ** 32), rng.randrange(1, 300), rng.randrange(2 ** 28, 2 ** 32)]))
        clients = sorted(cl, reverse=True)
        if nb > 1 and rng.random() < 0.05:
            rng.shuffle(clients)
        body = bytearray(vu(nb))
        end = {}
        for c in clients:
            clock = 0 if rng.random() < 0.8 else rng.randrange(1, 2 ** 20)
            ns = rng.choice([1, 1, 2, 3, 5, 10, 25, 40])
            b = bytearray()
            ck = clock
            for _s in range(ns):
                r = rng.random()
                if r < 0.55:
                    ln = rng.choice([1, 1, 1, 2, 3, 7, 20, 50, 63, 64, 65, 100, 200, 300])
                    txt = bytes(rng.choice(b"abcdefghij ") for _ in range(ln))
                    if rng.random() < 0.03:
                        txt = txt[:-1] + "\u00e9".encode()
                    shape = rng.random()
                    if shape < 0.5:
                        hdr = bytes([0xC4]) + vu(rng.choice(clients)) + vu(rng.randrange(400)) + vu(rng.choice(clients)) + vu(rng.randrange(400))
                    elif shape < 0.75:
                        hdr = bytes([0x84]) + vu(rng.choice(clients)) + vu(rng.randrange(400))
                    elif shape < 0.85:
                        hdr = bytes([0x44]) + vu(rng.choice(clients)) + vu(rng.randrange(400))
                    elif shape < 0.93:
                        sub = rng.random() < 0.4
                        hdr = bytes([0x24 if sub else 0x04]) + b"\x01" + vu(7) + b"default" + ((vu(3) + b"key") if sub else b"")
                    else:
                        hdr = bytes([0x04]) + b"\x00" + vu(rng.choice(clients)) + vu(rng.randrange(50))
                    b += hdr + vu(len(txt)) + txt
                    ck += len(txt.decode().encode("utf-16-le")) // 2
                elif r < 0.7:
                    n = rng.choice([1, 2, 9, 300, 70000])
                    b += bytes([0x81]) + vu(rng.choice(clients)) + vu(rng.randrange(400)) + vu(n)
                    ck += n
                elif r < 0.78:
                    n = rng.choice([1, 3, 40])
                    b += bytes([0x20 if rng.random() < 0.03 else 0x00]) + vu(n)
                    ck += n
                elif r < 0.84:
                    n = rng.choice([1, 5, 200])
                    b += bytes([10]) + vu(n)
                    ck += n
                elif r < 0.92:
                    if rng.random() < 0.5:
                        b += bytes([0x87]) + vu(rng.choice(clients)) + vu(rng.randrange(400)) + vu(3) + vu(9) + b"paragraph"
                    else:
                        b += bytes([0x87]) + vu(rng.choice(clients)) + vu(rng.randrange(400)) + vu(6)
                    ck += 1
                else:
                    raw = bytes(rng.randrange(256) for _ in range(rng.choice([0, 3, 80])))
                    b += bytes([0x83]) + vu(rng.choice(clients)) + vu(rng.randrange(400)) + vu(len(raw)) + raw
                    ck += 1
            body += vu(ns) + vu(c) + vu(clock) + b
            end[c] = ck
        nds = rng.choice([0, 0, 1, 2, 4])
        dcl = sorted({rng.randrange(1, 2 ** 32) for _ in range(nds)} | set(rng.sample(clients, min(len(clients), 1))) if nds else set(),
                     reverse=True)
        if len(dcl) > 1 and rng.random() < 0.1:
            rng.shuffle(dcl)
        body += vu(len(dcl))
        for c in dcl:
            nr = 0 if rng.random() < 0.03 else rng.choice([1, 1, 2, 5])
            body += vu(c) + vu(nr)
            for _r in range(nr):
                body += vu(rng.randrange(500)) + vu(rng.choice([1, 2, 30]))
        u = bytes(body)
        if rng.random() < 0.04 and len(u) > 1:
            u = u[:rng.randrange(1, len(u))]
        elif rng.random() < 0.03:
            u = u + b"\x07"
        docs.append(u)
        ends.append(end)
    return docs, ends


def _walker_svs(ends, seed):
    from v1util import vu
    rng = random.Random(seed)
    svs = []
    for end in ends:
        ents = [(c, rng.choice([0, e, max(e - 1, 0), rng.randrange(e + 1), e + 3])) for c, e in end.items() if rng.random() < 0.8]
        if rng.random() < 0.1:
            ents.append((rng.randrange(1, 2 ** 32), rng.randrange(100)))
        rng.shuffle(ents)
        if ents and rng.random() < 0.1:
            ents.append(ents[0])
        sv = vu(len(ents)) + b"".join(vu(c) + vu(k) for c, k in ents)
        if rng.random() < 0.02:
            sv += b"\x01"
        svs.append(sv)
    return svs


@pytest.mark.parametrize("env", [None, "YGM_WALK_GRID=3"])
def test_walker_states_vs_oracle(eng, env, monkeypatch):
    # the SV / diff ring walker on rich merged-state shapes; grid=3 gives every lane ~10 documents
    # (the per-round hand-over of documents, ring reuse across documents)
    if env:
        monkeypatch.setenv(*env.split("="))
    docs, ends = _walker_states(2000, seed=77)
    svs = _walker_svs(ends, seed=78)
    lean0 = eng.stats().docs_lean
    res = eng.encode_state_vector_from_update_batch(docs)
    bad = [d for d, u in enumerate(docs) if not same(oracle.encode_state_vector_from_update(u), res[d])]
    assert not bad, (len(bad), docs[bad[0]].hex())
    res = eng.diff_update_batch(docs, svs)
    bad = [d for d, u in enumerate(docs) if not same(oracle.diff_update(u, svs[d]), res[d])]
    assert not bad, (len(bad), docs[bad[0]].hex(), svs[bad[0]].hex())
    took = eng.stats().docs_lean - lean0
    assert len(docs) // 2 < took < 2 * len(docs)   # most documents stay on the walker, some defer


def _lean_ds_docs(n_docs, seed):
    """Debounce logs with deletions: struct updates (1-4 clients, clock-contiguous) mixed with
    delete-set-only updates and struct updates carrying a delete set.  The delete sets probe
    rule R-DS: several clients (in and outside the struct blocks), overlapping, adjacent,
    duplicate and zero-length ranges, clients without ranges, > 64 ranges per document,
    5-byte clients, clocks past 2^28, non-minimal varuints and truncated delete sets."""
    from v1util import vu, encode_ds
    rng = random.Random(seed)
    docs = []
    for _ in range(n_docs):
        ncl = rng.choice([1, 1, 2, 3, 4])
        clients = [rng.randrange(1, 2 ** 32) if rng.random() < 0.9 else rng.randrange(1, 100) for _ in range(ncl)]
        others = [rng.randrange(1, 2 ** 32) for _ in range(rng.choice([0, 1, 2, 5]))]
        clocks = [0] * ncl
        big = rng.random() < 0.04
        many = rng.random() < 0.04
        ups = []
        for _ in range(rng.randrange(2, 80)):
            r = rng.random()
            if r < 0.6 or not ups:
                c = rng.randrange(ncl)
                txt = "".join(rng.choice("xyz") for _ in range(rng.choice([1, 1, 2, 4])))
                body = bytes([0x84]) + vu(clients[c]) + vu(max(clocks[c], 1) - 1) + vu(len(txt)) + txt.encode()
                if clocks[c] == 0:
                    body = bytes([4]) + b"\x01" + vu(1) + b"t" + vu(len(txt)) + txt.encode()
                u = vu(1) + vu(1) + vu(clients[c]) + vu(clocks[c]) + body
                clocks[c] += len(txt)
                ds = [] if rng.random() < 0.85 else None
            else:
                u = b"\x00"
                ds = None
            if ds is None:   # a delete set
                pool = clients + others
                ds = []
                for cl in rng.sample(pool, min(len(pool), rng.choice([1, 1, 1, 2, 3]))):
                    rs = []
                    for _r in range(rng.choice([1, 1, 2, 3] + ([12] if many else []))):
                        ck = rng.randrange(2 ** 29, 2 ** 30) if big and rng.random() < 0.3 else rng.randrange(0, 60)
                        ln = rng.choice([1, 1, 2, 5]) if rng.random() < 0.97 else 0
                        rs.append((ck, ln))
                    if rng.random() < 0.02:
                        rs = []                                   # a client without ranges
                    ds.append((cl, rs))
            e = encode_ds(ds)
            if rng.random() < 0.02 and len(e) > 2:
                e = e[:-1] + bytes([e[-1] | 0x80, 0])              # non-minimal last varuint
            if rng.random() < 0.001:
                e = e[:-1]                                         # truncated: yjs throws
            ups.append(u + e)
        docs.append(ups)
    return docs


def test_lean_kernel_delete_sets_vs_oracle(eng):
    docs = _lean_ds_docs(1500, seed=606)
    lean0 = eng.stats().docs_lean
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), [u.hex() for u in docs[bad[0]]])
    took = eng.stats().docs_lean - lean0
    assert len(docs) // 10 < took < len(docs)   # both paths (updates > 32 bytes defer)


def test_lean_kernel_delete_sets_compat135_vs_oracle(eng, eng135):
    # yjs 13.5 writes delete-set clients in first-seen order (mergeDeleteSets' Map insertion order): the lean, wave
    # and workgroup tiers order the union's clients by their least (update, range) rank -- the 13.5 mode sends no
    # more documents to the sequential kernel than the 13.6 mode does (> 64 ranges: the wave tier; > 128: the
    # workgroup tier)
    docs = _lean_ds_docs(1500, seed=607)
    st0 = eng135.stats()
    res = eng135.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us, compat135=True), res[d])]
    assert not bad, (len(bad), [u.hex() for u in docs[bad[0]]])
    st1 = eng135.stats()
    s0 = eng.stats().docs_seq
    eng.merge_updates_batch(docs)
    assert st1.docs_seq - st0.docs_seq == eng.stats().docs_seq - s0
    assert st1.docs_fast - st0.docs_fast > 0 and st1.docs_lean - st0.docs_lean > len(docs) // 10


def test_compat135_multi_client_c2_deletions_stay_parallel(eng135):
    # C2 logs of 2-4 clients with 20 % deletions under yjs 13.5 -- multi-client delete-set unions in
    # first-seen client order, bit-exact, and not one document on the sequential kernel
    from tools import synth
    arena, upd_off, doc_upd = synth.text_updates(2000, 200, min_clients=2, max_clients=4, del_pct=20, seed=135)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(2000)]
    st0 = eng135.stats()
    res = eng135.merge_updates_batch(docs)
    st1 = eng135.stats()
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us, compat135=True), res[d])]
    assert not bad, (len(bad), bad[:5])
    assert st1.docs_seq - st0.docs_seq == 0
    # the 13.5 order is not the 13.6 one on most of these documents (the test would not see a wrong order otherwise)
    differ = sum(oracle.merge_updates(us, compat135=True) != oracle.merge_updates(us) for us in docs[:200])
    assert differ > 50


def test_compat135_large_documents_vs_oracle(eng135):
    # the large-document tier unions delete sets in client-descending order only (its splice walks U0's
    # canonical delete set); under yjs 13.5 a document whose merged delete set has several clients goes on to the
    # sequential kernel (first-seen order, bit-exact) -- a stated limit, measured here: every document
    # is the oracle's, and each is finished by the large-document tier or by the sequential kernel
    from tools import synth
    arena, upd_off, doc_upd = synth.big_docs(12, 200000, 16 * 1024, max_clients=64, max_k=60, seed=136)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(12)]
    st0 = eng135.stats()
    res = eng135.merge_updates_batch(docs)
    st1 = eng135.stats()
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us, compat135=True), res[d])]
    assert not bad, (len(bad), bad[:5])
    n_seq, n_big = st1.docs_seq - st0.docs_seq, st1.docs_big - st0.docs_big
    assert n_seq + n_big == len(docs) and n_seq > 0, (n_seq, n_big)


@pytest.mark.parametrize("xml", [False, True])
def test_large_documents_c3_c5_vs_oracle(eng, xml):
    # SURVEY.md §8d C3 / C5 shapes at test size: Zipf-sized [snapshot, ...log] documents (GC,
    # deleted content, merged delete sets, 40 % deletions in the log) and XmlFragment snapshots
    # over thousands of client blocks -- the workgroup and sequential tiers, bit-exact
    from tools import synth
    if xml:
        arena, upd_off, doc_upd = synth.big_docs(4, 400000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=4)
    else:
        arena, upd_off, doc_upd = synth.big_docs(60, 300000, 1024, max_clients=64, max_k=200, seed=3)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(len(doc_upd) - 1)]
    st0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), bad[:5])
    assert all(st == 0 for st, _ in res)
    if xml:   # XmlElement attributes (ContentAny map entries) are in the snapshots and the large-document tier takes them
        assert all(us[0].count(bytes([0x28, 0x00])) > 100 for us in docs)
        assert eng.stats().docs_seq - st0.docs_seq == 0


def test_large_documents_live_sessions_vs_oracle(eng):
    # [state, ...log] documents of simulated sessions yjs integrates (tools/synth_live.c): Tiptap-style XmlFragment
    # states hold overwritten attributes -- map entries written with an origin AND the parentSub bit 0x20 (info 0xA8),
    # which yjs's merge writes back without the bit -- and Y.Text states with strings split by later inserts.  The
    # large-document tier takes them (the bit cleared by its copies: big_validate marks them in the scan's bitmap),
    # bit-exact against the oracle; the sequential kernel takes none.
    from tools import synth
    docs = []
    for n, mb, kw in ((4, 700000, dict(min_bytes=64 * 1024, n_clients=10000, xml=True, max_k=50, seed=15)),
                      (6, 300000, dict(min_bytes=8 * 1024, n_clients=300, xml=True, max_k=30, seed=16)),
                      (8, 400000, dict(min_bytes=4 * 1024, n_clients=64, max_k=200, seed=17))):
        a, uo, du = synth.live_docs(n, mb, **kw)
        ups = synth.split(a, uo)
        docs += [ups[du[d]:du[d + 1]] for d in range(n)]
    assert sum(us[0].count(bytes([0xA8])) > 10 for us in docs[:10]) >= 8   # (a lower bound: 0xA8 bytes elsewhere too)
    st0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), bad[:5])
    s1 = eng.stats()
    assert s1.docs_seq - st0.docs_seq == 0 and s1.docs_big - st0.docs_big == len(docs), (s1.docs_seq - st0.docs_seq, s1.docs_big - st0.docs_big)


def _log_structs(us):
    # struct count of a document's log (every update but the largest): the block headers' counts
    def vu(b, p):
        n = s = 0
        while True:
            c = b[p]; p += 1; n |= (c & 127) << s; s += 7
            if c < 128:
                return n, p
    i0 = max(range(len(us)), key=lambda i: len(us[i]))
    t = 0
    for i, u in enumerate(us):
        if i == i0:
            continue
        nb, p = vu(u, 0)
        assert nb <= 1   # (synth: one block per log update)
        if nb:
            t += vu(u, p)[0]
    return t


def test_large_documents_mid_and_large_sizes_vs_oracle(eng):
    # the mid-size kernel holds 256 log structs / delete ranges in LDS; documents over that go on to the large size
    from tools import synth
    arena, upd_off, doc_upd = synth.big_docs(8, 300000, 1024, max_clients=64, max_k=900, seed=5)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(8)]
    counts = [_log_structs(us) for us in docs]
    assert sum(c > 256 for c in counts) >= 3 and sum(c <= 256 for c in counts) >= 2, counts
    st0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (bad, counts)
    assert eng.stats().docs_big - st0.docs_big == len(docs)


def test_large_document_10mb_vs_oracle(eng):
    # BASELINE C3's largest size: one 10 MB [snapshot, ...log] document through the large-document tier
    from tools import synth
    arena, upd_off, doc_upd = synth.big_docs(1, 10_000_000, 1024, max_clients=64, max_k=200, seed=9)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[0]:doc_upd[1]]]
    assert len(docs[0][0]) > 9_000_000
    st0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    assert same(oracle.merge_updates(docs[0]), res[0])
    assert res[0][0] == 0 and eng.stats().docs_big - st0.docs_big == 1


def test_large_document_tile_edges_vs_oracle(eng):
    from tile_docs import tile_edge_docs
    docs = tile_edge_docs(5)
    for us in docs:
        assert len(us[0]) > 16384
        assert oracle.merge_updates(us)[0] == 0
    st0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, bad
    assert eng.stats().docs_big - st0.docs_big == len(docs)   # the large-document tier took every one


def test_large_document_delete_set_splice_vs_oracle(eng):
    # snapshot delete sets large against the log's ranges are spliced (the snapshot's entries copied as written, log
    # ranges merged in by binary search); broken snapshot delete sets (adjacent, overlapping, empty, non-minimal) are
    # streamed instead -- bit-exact either way, every document in the large-document tier
    from tile_docs import ds_splice_docs
    docs = [us for seed in (11, 12, 13) for us in ds_splice_docs(seed)]
    st0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, (len(bad), bad[:5])
    assert eng.stats().docs_big - st0.docs_big == len(docs)


def test_large_document_unsorted_delete_set_goes_on(eng):
    # a snapshot delete set outside union order: the large-document tier's first emit pass refuses it and
    # the sequential kernel merges it, bit-exact
    from tile_docs import tile_edge_docs
    docs = tile_edge_docs(6, ds_ascending=True)
    st0 = eng.stats()
    res = eng.merge_updates_batch(docs)
    bad = [d for d, us in enumerate(docs) if not same(oracle.merge_updates(us), res[d])]
    assert not bad, bad
    st1 = eng.stats()
    assert st1.docs_big - st0.docs_big == 0 and st1.docs_seq - st0.docs_seq == len(docs)


def test_sharded_engine_two_contexts_match_single(eng):
    # SURVEY.md §8e in one process: two engine contexts (the box has one GPU) behind fnv1a64 routing
    from hocuspocus_amd.shard import ShardedEngine
    from tools import synth
    arena, upd_off, doc_upd = synth.text_updates(300, 60, seed=12, del_pct=10)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(300)]
    names = [f"doc-{d}" for d in range(300)]
    se = ShardedEngine(devices=(0, 0))
    try:
        got = se.merge_updates_batch(names, docs)
        merged = [m for _, m in got]
        svs = se.encode_state_vector_from_update_batch(names, merged)
        diffs = se.diff_update_batch(names, merged, [b"\x00"] * len(merged))
    finally:
        se.close()
    assert got == eng.merge_updates_batch(docs)
    assert svs == eng.encode_state_vector_from_update_batch(merged)
    assert all(d == (0, m) for d, m in zip(diffs, merged))
