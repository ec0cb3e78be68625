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
