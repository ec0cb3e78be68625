"""SyncStep2 wire parity: the reference answers a SyncStep1 with
Y.encodeStateAsUpdate(doc, sv) of the live document (packages/server/src/MessageReceiver.ts:137-138).  For a
document loaded from stored bytes u (Database.ts:44-50) that is encodeStateAsUpdate(applyUpdate(new Doc, u), sv).

It equals diffUpdate(snapshot(u), sv) -- the f-1 snapshot, then a diff -- except for one bit: Item.write of an
integrated item sets info bit 0x20 whenever parentSub !== null (Y@80416), while diffUpdate's lazy reader drops
it beside an origin.  The responder therefore diffs the snapshot with every struct keeping its input's bit
(YGM_F_KEEP_SUB / the oracle's YO_KEEP_SUB), ygm_sync_step2_v1.

Pinned by tests/golden/step2_v135.json.gz (tools/step2_corpus.js: the yjs 13.5.16 bundle's own
encodeStateAsUpdate(doc, sv) over the 760 f-1 sessions x three state vectors; 33 rows where 13.5's writeString
throws on a cut surrogate pair are null)."""
import gzip
import json
import os
import shutil
import subprocess

import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "step2_v135.json.gz")
SNAPS = [os.path.join(ROOT, "tests", "golden", f) for f in ("snapshot_v135.json.gz", "snapshot_text_v135.json.gz")]
NODE = shutil.which("node")
BUNDLE = os.path.exists("/opt/conda/share/jupyter/lab/static/3502.fbe0c610be82ba1360db.js")


def rows():
    d = json.load(gzip.open(FIX, "rt"))
    return [(bytes.fromhex(u), bytes.fromhex(sv), None if e is None else bytes.fromhex(e), eq) for u, sv, e, eq in d["rows"]]


def yjs_snapshots():
    """state -> yjs 13.5.16 encodeStateAsUpdate(applyUpdate(new Doc, state)) from the f-1 fixtures"""
    out = {}
    for f in SNAPS:
        for u, e in json.load(gzip.open(f, "rt"))["rows"]:
            out[bytes.fromhex(u)] = bytes.fromhex(e)
    return out


def test_step2_fixtures_present():
    r = rows()
    assert len(r) == 2280
    assert sum(1 for *_, e, _eq in r if e is None) == 33
    assert sum(eq for *_, eq in r) == 1713   # diffUpdate alone matches only where no struct keeps the bit


@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle (image) needed")
def test_step2_fixtures_regenerate(tmp_path):
    out = str(tmp_path / "s2.json.gz")
    subprocess.run([NODE, os.path.join(ROOT, "tools", "step2_corpus.js"), out], check=True, timeout=600, capture_output=True)
    assert json.load(gzip.open(out, "rt"))["rows"] == json.load(gzip.open(FIX, "rt"))["rows"]


def test_oracle_step2_is_keep_sub_diff_of_snapshot():
    """encodeStateAsUpdate(doc, sv) == diff(snapshot, sv, keep parentSub bits), byte for byte, on every row (13.5)"""
    snaps = yjs_snapshots()
    bad = []
    for k, (u, sv, exp, _eq) in enumerate(rows()):
        st, got = oracle.diff_update(snaps[u], sv, compat135=True, keep_sub=True)
        if exp is None:
            if st != 4:   # YO_ESURROGATE: 13.5's writeString throws on the lone surrogate
                bad.append(k)
        elif (st, got) != (0, exp):
            bad.append(k)
    assert not bad, f"{len(bad)} rows differ, first {bad[:5]}"


def test_oracle_plain_diff_differs_only_by_the_bit():
    """the fixture's 4th column: plain diffUpdate(snapshot, sv) equals the reply exactly where it says so"""
    snaps = yjs_snapshots()
    for u, sv, exp, eq in rows()[:600]:
        st, got = oracle.diff_update(snaps[u], sv, compat135=True)
        if exp is None:
            continue
        assert (st == 0 and got == exp) == bool(eq)
        if not eq:
            assert len(got) == len(exp) and all((a ^ b) in (0, 0x20) for a, b in zip(got, exp))


@pytest.fixture(scope="module")
def eng135():
    from hocuspocus_amd import Engine
    e = Engine(0, compat135=True)
    yield e
    e.close()


@pytest.mark.gpu
def test_gpu_step2_vs_yjs(eng135):
    """ygm_sync_step2_v1 (GPU snapshot of the stored state + keep-parentSub diff) == yjs encodeStateAsUpdate(doc, sv)"""
    r = rows()
    res = eng135.sync_step2_batch([u for u, *_ in r], [sv for _, sv, *_ in r])
    bad = []
    for k, ((u, sv, exp, _), got) in enumerate(zip(r, res)):
        if exp is None:
            if got[0] != 4:
                bad.append(k)
        elif got != (0, exp):
            bad.append(k)
    assert not bad, f"{len(bad)} replies differ from yjs, first {bad[:5]}: {res[bad[0]]}"


@pytest.mark.gpu
def test_gpu_step2_default_mode_vs_oracle():
    """13.6 default mode: GPU replies vs the oracle's keep-sub diff of the GPU-checked snapshot (default mode)"""
    from hocuspocus_amd import Engine
    r = rows()
    with Engine(0) as e:
        snaps = e.snapshot_batch([u for u, *_ in r])
        res = e.sync_step2_batch([u for u, *_ in r], [sv for _, sv, *_ in r])
    bad = []
    for k, ((u, sv, *_), (sst, snap), got) in enumerate(zip(r, snaps, res)):
        assert sst == 0
        if got != oracle.diff_update(snap, sv, keep_sub=True):
            bad.append(k)
    assert not bad, f"{len(bad)} differ, first {bad[:5]}"


# ---------------------------------------------------------------------------------------- states with lost updates
# tests/golden/step2_pending_v135.json.gz (node tools/step2_corpus.js OUT pending): the states of the pending and
# sub-document snapshot corpora, pending ones kept, x four state vectors (empty, a cut, the store's own, the state's
# own -- past the store's, inside the pending structs).  yjs's reply is mergeUpdates([writeStateAsUpdate(doc, sv),
# pendingDs, diffUpdate(pending structs, sv)]) (Y@23300): the state part keeps each struct's parentSub bit, the
# pending structs are diffed by the lazy writer's rules.
PFIX = os.path.join(ROOT, "tests", "golden", "step2_pending_v135.json.gz")


def pending_rows():
    d = json.load(gzip.open(PFIX, "rt"))
    return [(bytes.fromhex(u), bytes.fromhex(sv), None if e is None else bytes.fromhex(e)) for u, sv, e, _eq in d["rows"]]


def test_step2_pending_fixtures_present():
    r = pending_rows()
    assert len(r) == 2320 and sum(1 for *_, e in r if e is None) == 22


@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle (image) needed")
def test_step2_pending_fixtures_regenerate(tmp_path):
    out = str(tmp_path / "s2p.json.gz")
    subprocess.run([NODE, os.path.join(ROOT, "tools", "step2_corpus.js"), out, "pending"], check=True, timeout=600, capture_output=True)
    assert json.load(gzip.open(out, "rt"))["rows"] == json.load(gzip.open(PFIX, "rt"))["rows"]


def _parts_reply(body, st, sv, compat135):
    """The reply from the kernel code's output: a complete state's snapshot diffed keeping the bit; a pending one's
    three parts (PendHdr) diffed (state: keeping the bit, pending structs: plain) and merged -- the engine's steps."""
    import struct
    if st == 0:
        return oracle.diff_update(body, sv, compat135=compat135, keep_sub=True)
    assert st == 64
    ln = struct.unpack_from("<IIII", body, 0)
    a, b, c = body[16:16 + ln[0]], body[16 + ln[0]:16 + ln[0] + ln[1]], body[16 + ln[0] + ln[1]:16 + ln[0] + ln[1] + ln[2]]
    sa, da = oracle.diff_update(a, sv, compat135=compat135, keep_sub=True)
    sc, dc = oracle.diff_update(c, sv, compat135=compat135)
    if sa or sc:
        return (sa or sc), None
    return oracle.merge_updates([da, b, dc], compat135=compat135)


def _kernel_outputs(tmp_path, states, mode):
    from test_snapshot import write_in, read_res
    exe = str(tmp_path / "snapdev")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "snapdev", "snapdev.cpp")], check=True, timeout=300)
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_in(a, states)
    subprocess.run([exe, a, b, str(mode)], check=True, timeout=120)
    return read_res(b)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_step2_pending_decomposition_on_host(tmp_path):
    """The engine's decomposition, with the snapshot kernel's code host-compiled and the oracle's diff / merge, gives
    yjs's reply on every row (13.5); where 13.5 throws (a cut surrogate pair) a part's diff refuses."""
    r = pending_rows()
    uniq = list(dict.fromkeys(u for u, *_ in r))
    outs = dict(zip(uniq, _kernel_outputs(tmp_path, uniq, 1)))
    assert sum(st == 64 for st, _ in outs.values()) >= 200
    bad = []
    for k, (u, sv, exp) in enumerate(r):
        st, body = outs[u]
        got = _parts_reply(body, st, sv, True)
        if exp is None:
            if got[0] != 4:
                bad.append(k)
        elif got != (0, exp):
            bad.append(k)
    assert not bad, f"{len(bad)} rows differ, first {bad[:5]}"


@pytest.mark.gpu
def test_gpu_step2_pending_vs_yjs(eng135):
    """ygm_sync_step2_v1 on states with lost updates (the pending parts split off, diffed on child contexts, merged)
    == yjs encodeStateAsUpdate(doc, sv), mixed with complete states."""
    r = pending_rows() + [(u, sv, e) for u, sv, e, _ in rows()[:300]]
    res = eng135.sync_step2_batch([u for u, *_ in r], [sv for _, sv, _ in r])
    bad = []
    for k, ((u, sv, exp), got) in enumerate(zip(r, res)):
        if exp is None:
            if got[0] != 4:
                bad.append(k)
        elif got != (0, exp):
            bad.append(k)
    assert not bad, f"{len(bad)} replies differ from yjs, first {bad[:5]}: {res[bad[0]]}"


@pytest.mark.gpu
@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_gpu_step2_pending_default_mode_vs_oracle(tmp_path):
    """13.6 default mode: GPU replies vs the decomposition over the host-compiled kernel code and the oracle (default)."""
    from hocuspocus_amd import Engine
    r = pending_rows()[:1200]
    uniq = list(dict.fromkeys(u for u, *_ in r))
    outs = dict(zip(uniq, _kernel_outputs(tmp_path, uniq, 0)))
    with Engine(0) as e:
        res = e.sync_step2_batch([u for u, *_ in r], [sv for _, sv, _ in r])
    bad = [k for k, ((u, sv, _), got) in enumerate(zip(r, res)) if got != _parts_reply(outs[u][1], outs[u][0], sv, False)]
    assert not bad, f"{len(bad)} differ, first {bad[:5]}"
