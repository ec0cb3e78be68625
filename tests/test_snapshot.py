"""Doc-normalized snapshot: snapshot(u) = Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), u)).

The checker is yjs itself -- the image's 13.5.16 bundle (tools/yjs_bundle.js) -- through
  * tests/golden/snapshot_v135.json.gz: 440 multi-peer editing sessions (tools/snap_corpus.js: Y.Text with
    UTF-8 of every width, formatting, embeds, Y.Array / Y.Map with nested types and overwrites, XmlFragment
    trees with attributes, deleted nested types, concurrent peers) and their yjs snapshots;
  * live sessions generated on the GPU box by the same script with fresh seeds (Node + the bundle ship in
    the image there too);
  * the GPU merge's own outputs for C2 logs, snapshotted by yjs (tools/snap_expect.js).
CPU tests pin the fixtures (regenerated here by the committed generator) and run the kernel's sequential
code (ygm_snapshot.hpp) host-compiled through tools/snapdev; GPU tests run the HIP kernel through the C ABI
in 13.5 compat mode (the bundle's behaviour).  The 13.6 default writes the delete set's clients in descending
order instead of store order (the only difference in a snapshot's bytes): the default mode is
pinned against the same yjs vectors with their delete sets rewritten client-descending (golden.ds_to_desc) --
a derived expectation, as no 13.6 yjs is in the image."""
import gzip
import json
import os
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "snapshot_v135.json.gz")
NODE = shutil.which("node")
BUNDLE = os.path.exists("/opt/conda/share/jupyter/lab/static/3502.fbe0c610be82ba1360db.js")


def fixtures():
    d = json.load(gzip.open(FIX, "rt"))
    return [(bytes.fromhex(u), bytes.fromhex(e)) for u, e in d["rows"]]


def write_in(path, us):
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(us)))
        for u in us:
            f.write(struct.pack("<I", len(u)))
            f.write(u)


def read_res(path):
    b = open(path, "rb").read()
    i, out = 0, []
    while i < len(b):
        st, ln = struct.unpack_from("<iI", b, i)
        i += 8
        out.append((st, b[i:i + ln]))
        i += ln
    return out


def read_in(path):
    b = open(path, "rb").read()
    n = struct.unpack_from("<I", b, 0)[0]
    i, out = 4, []
    for _ in range(n):
        ln = struct.unpack_from("<I", b, i)[0]
        i += 4
        out.append(b[i:i + ln])
        i += ln
    return out


def test_fixtures_present():
    rows = fixtures()
    assert len(rows) == 440 and all(u and e for u, e in rows)


@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle are needed to regenerate")
def test_fixtures_regenerate(tmp_path):
    """The committed vectors are what the committed generator produces from the bundle (first sessions)."""
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "exp.bin")
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_corpus.js"), "20", "11", a, b, "80"], check=True, timeout=120)
    rows = fixtures()[:20]
    assert read_in(a) == [u for u, _ in rows]
    assert [e for _, e in read_res(b)] == [e for _, e in rows]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_kernel_code_on_host_vs_fixtures(tmp_path):
    """The kernel's sequential code (ygm_snapshot.hpp), host-compiled, against the yjs vectors (13.5 mode)."""
    exe = str(tmp_path / "snapdev")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "snapdev", "snapdev.cpp")], check=True, timeout=300)
    rows = fixtures()
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_in(a, [u for u, _ in rows])
    subprocess.run([exe, a, b, "1"], check=True, timeout=120)
    got = read_res(b)
    assert [g for g in got] == [(0, e) for _, e in rows]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_kernel_code_on_host_default_mode(tmp_path):
    """The same host-compiled kernel code in the 13.6 default mode: the yjs vectors with client-descending delete sets."""
    from golden import ds_to_desc
    exe = str(tmp_path / "snapdev")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "snapdev", "snapdev.cpp")], check=True, timeout=300)
    rows = fixtures()
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_in(a, [u for u, _ in rows])
    subprocess.run([exe, a, b, "0"], check=True, timeout=120)
    got = read_res(b)
    assert got == [(0, bytes.fromhex(ds_to_desc(e.hex()))) for _, e in rows]


def _live_batch(specs):
    """[state, ...log] documents of simulated sessions (tools/synth_live.c), merged by the oracle: (merged states, their
    first updates alone) -- what GpuMerge snapshots."""
    import oracle
    from tools import synth
    out = []
    for n, max_bytes, kw in specs:
        a, uo, du = synth.live_docs(n, int(max_bytes), **kw)
        ups = synth.split(a, uo)
        for d in range(n):
            st, m = oracle.merge_updates(ups[du[d]:du[d + 1]])
            assert st == 0
            out.append(m)
            out.append(ups[du[d]])
    return out


LIVE_SPECS = ((6, 5e4, dict(min_bytes=2000, n_clients=300, xml=True, seed=21)), (6, 5e4, dict(min_bytes=2000, n_clients=8, seed=22)),
              (20, 2e4, dict(min_bytes=2000, n_clients=40, xml=True, seed=23, max_k=10)),
              (10, 1e4, dict(min_bytes=2000, n_clients=3, seed=24, max_k=30)))


@pytest.mark.skipif(not (NODE and BUNDLE) or shutil.which("g++") is None, reason="node + the yjs bundle and a host compiler needed")
def test_kernel_code_on_host_vs_yjs_live_docs(tmp_path):
    """Live-session documents (tools/synth_live.c: Tiptap-style XmlFragment trees with formats, embeds, attributes and
    up to 300 clients; Y.Text with heavy deletions and strings split by later inserts), merged by the oracle, snapshotted
    by yjs and by the kernel's code host-compiled -- 13.5 mode, and the 13.6 default against the client-descending
    rewrite.  Every document integrates completely in yjs (no pending structs)."""
    from golden import ds_to_desc
    exe = str(tmp_path / "snapdev")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "snapdev", "snapdev.cpp")], check=True, timeout=300)
    us = _live_batch(LIVE_SPECS)
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "exp.bin")
    write_in(a, us)
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_expect.js"), a, b], check=True, timeout=240)
    exp = read_res(b)
    assert all(st == 0 for st, _ in exp)
    for mode in ("1", "0"):
        g = str(tmp_path / f"got{mode}.bin")
        subprocess.run([exe, a, g, mode], check=True, timeout=120)
        want = exp if mode == "1" else [(0, bytes.fromhex(ds_to_desc(e.hex()))) for _, e in exp]
        got = read_res(g)
        bad = [k for k in range(len(us)) if got[k] != want[k]]
        assert not bad, f"mode {mode}: {len(bad)} differ, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle (image) needed")
def test_gpu_snapshot_at_baseline_sizes(eng135, tmp_path):
    """f-1 at the sizes BASELINE configs C5 / C3 name: 4 Tiptap-style documents of 10 000 client
    blocks (0.4-1 MB) and 2 Y.Text documents over 1 MB with heavy deletions, [state, ...log] of live sessions
    (tools/synth_live.c), merged on the GPU (against the oracle), then snapshotted on the GPU, against yjs's
    snapshot of the merge."""
    import oracle
    from tools import synth
    docs = []
    for n, mb, kw in ((4, 1.0e6, dict(min_bytes=64 * 1024, n_clients=10000, xml=True, max_k=50, seed=5)),
                      (2, 2.2e6, dict(min_bytes=1 << 20, n_clients=64, max_k=200, seed=3))):
        a, uo, du = synth.live_docs(n, int(mb), **kw)
        ups = synth.split(a, uo)
        docs += [ups[du[d]:du[d + 1]] for d in range(n)]
    merged = eng135.merge_updates_batch(docs)
    assert merged == [oracle.merge_updates(d, compat135=True) for d in docs]
    states = [m for _, m in merged]
    assert sum(len(m) >= 1 << 20 for m in states) >= 2
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "exp.bin")
    write_in(a, states)
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_expect.js"), a, b], check=True, timeout=240)
    exp = read_res(b)
    assert all(st == 0 for st, _ in exp)
    got = eng135.snapshot_batch(states)
    bad = [k for k in range(len(states)) if got[k] != exp[k]]
    assert not bad, f"{len(bad)} differ, first {bad[:3]}: {[got[k][0] for k in bad[:3]]}"
    # smaller live sessions (every client count, both root types) in one more batch
    us = _live_batch(LIVE_SPECS)
    write_in(a, us)
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_expect.js"), a, b], check=True, timeout=240)
    assert eng135.snapshot_batch(us) == read_res(b)


# ---------------------------------------------------------------------------------------- flat text (k_snap_text)
TFIX = os.path.join(ROOT, "tests", "golden", "snapshot_text_v135.json.gz")


def text_fixtures():
    d = json.load(gzip.open(TFIX, "rt"))
    return [(bytes.fromhex(u), bytes.fromhex(e)) for u, e in d["rows"]]


def test_text_fixtures_present():
    rows = text_fixtures()
    assert len(rows) == 320 and all(u and e for u, e in rows)


@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle are needed to regenerate")
def test_text_fixtures_regenerate(tmp_path):
    """The committed flat-text vectors are what the generator's text mode produces from the bundle (first sessions)."""
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "exp.bin")
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_corpus.js"), "30", "21", a, b, "150", "text"], check=True, timeout=120)
    rows = text_fixtures()[:30]
    assert read_in(a) == [u for u, _ in rows]
    assert [e for _, e in read_res(b)] == [e for _, e in rows]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("mode", [1, 0])
def test_text_kernel_code_on_host(tmp_path, mode):
    """The flat-text snapshot (ygm_snap_text.hpp, k_snap_text's code) host-compiled: on every document it takes
    (the 320 text sessions: concurrent peers, splits by origins and delete ranges; the 440 general sessions: the
    few that are flat text) its bytes are yjs's (13.5 mode; 13.6 default: client-descending delete sets) and the
    general kernel code's; documents it leaves (nested types, formats, non-ASCII, past a 6 KiB workspace) go to the general path."""
    from golden import ds_to_desc
    exe = str(tmp_path / "snaptext")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "snapdev", "snaptext.cpp")], check=True, timeout=300)
    for rows, min_taken in ((text_fixtures(), 300), (fixtures(), 1)):
        a, b = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
        write_in(a, [u for u, _ in rows])
        r = subprocess.run([exe, a, str(mode), "6144", b], check=True, timeout=120, capture_output=True, text=True)
        lines = [tuple(map(int, x.split())) for x in r.stdout.split("\n") if x]
        taken = [k for k, (t, _, _) in enumerate(lines) if t]
        assert len(taken) >= min_taken
        assert all(lines[k][2] == 1 for k in taken), "text path differs from the general kernel code"
        got = read_res(b)
        for k in taken:
            exp = rows[k][1] if mode else bytes.fromhex(ds_to_desc(rows[k][1].hex()))
            assert got[k] == (0, exp), f"document {k} differs from yjs"


# ---------------------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def eng135():
    from hocuspocus_amd import Engine
    e = Engine(0, compat135=True)
    yield e
    e.close()


@pytest.mark.gpu
def test_gpu_snapshot_vs_yjs_fixtures(eng135):
    rows = fixtures()
    res = eng135.snapshot_batch([u for u, _ in rows])
    bad = [k for k, ((_, e), r) in enumerate(zip(rows, res)) if r != (0, e)]
    assert not bad, f"{len(bad)} documents differ from yjs, first {bad[:5]}: {res[bad[0]]}"


@pytest.mark.gpu
def test_gpu_snapshot_default_mode_vs_fixtures():
    """The 13.6 default mode (what GpuMerge({normalize}) ships): the yjs vectors with client-descending delete sets."""
    from golden import ds_to_desc
    from hocuspocus_amd import Engine
    rows = fixtures()
    with Engine(0) as e:
        res = e.snapshot_batch([u for u, _ in rows])
    exp = [(0, bytes.fromhex(ds_to_desc(x.hex()))) for _, x in rows]
    bad = [k for k in range(len(rows)) if res[k] != exp[k]]
    assert not bad, f"{len(bad)} documents differ, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle (image) needed for live sessions")
def test_gpu_snapshot_vs_live_yjs(eng135, tmp_path):
    """Fresh sessions generated on this box by yjs, longer ones included."""
    for seed, n, ops in ((901, 300, 60), (902, 40, 1500)):
        a, b = str(tmp_path / f"in{seed}.bin"), str(tmp_path / f"exp{seed}.bin")
        subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_corpus.js"), str(n), str(seed), a, b, str(ops)], check=True, timeout=240)
        us, exp = read_in(a), read_res(b)
        res = eng135.snapshot_batch(us)
        bad = [k for k, (e, r) in enumerate(zip(exp, res)) if r != e]
        assert not bad, f"seed {seed}: {len(bad)} differ, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle (image) needed")
def test_gpu_snapshot_of_gpu_merges(eng135, tmp_path):
    """C2 debounce logs merged on the GPU, then snapshotted on the GPU, against yjs's snapshot of the merge."""
    from tools import synth
    arena, upd_off, doc_upd = synth.text_updates(300, 200, seed=41, del_pct=20)
    docs = [[arena[upd_off[u]:upd_off[u + 1]].tobytes() for u in range(doc_upd[d], doc_upd[d + 1])] for d in range(300)]
    merged = [m for st, m in eng135.merge_updates_batch(docs)]
    assert all(m is not None for m in merged)
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "exp.bin")
    write_in(a, merged)
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_expect.js"), a, b], check=True, timeout=240)
    assert eng135.snapshot_batch(merged) == [(st, e if st == 0 else None) for st, e in read_res(b)]


@pytest.mark.gpu
def test_gpu_snapshot_text_vs_yjs(eng135):
    """The flat-text sessions (k_snap_text for all but the largest) against yjs, both modes."""
    from golden import ds_to_desc
    from hocuspocus_amd import Engine
    rows = text_fixtures()
    res = eng135.snapshot_batch([u for u, _ in rows])
    bad = [k for k, ((_, e), r) in enumerate(zip(rows, res)) if r != (0, e)]
    assert not bad, f"{len(bad)} documents differ from yjs, first {bad[:5]}"
    with Engine(0) as e:
        res = e.snapshot_batch([u for u, _ in rows])
    bad = [k for k, ((_, x), r) in enumerate(zip(rows, res)) if r != (0, bytes.fromhex(ds_to_desc(x.hex())))]
    assert not bad, f"default mode: {len(bad)} documents differ, first {bad[:5]}"


@pytest.mark.gpu
def test_gpu_snapshot_lds_tier_equals_general(monkeypatch):
    """k_snap_text (flat text, input + workspace in LDS) against the count / scan / k_snap path alone
    (YGM_SNAP_NOLDS), on one batch mixing what each takes: the yjs vectors (nested types, splits), C2 merges with
    deletions, documents too large for the LDS tier (3 000-update logs, > 32 KB) and malformed / pending inputs."""
    from hocuspocus_amd import Engine
    from tools import synth
    with Engine(0, compat135=True) as e:
        batch = [u for u, _ in fixtures()]
        for n, k, seed in ((200, 200, 43), (4, 3000, 44)):
            arena, upd_off, doc_upd = synth.text_updates(n, k, seed=seed, del_pct=20)
            docs = [[arena[upd_off[u]:upd_off[u + 1]].tobytes() for u in range(doc_upd[d], doc_upd[d + 1])] for d in range(n)]
            batch += [m for st, m in e.merge_updates_batch(docs)]
        assert max(len(u) for u in batch) > 40000
        batch += [b"", bytes([1, 1, 5, 3, 0x04, 1, 1, 0x74, 1, 0x61, 0]), batch[3][:len(batch[3]) // 2]]
        got = e.snapshot_batch(batch)
        monkeypatch.setenv("YGM_SNAP_NOLDS", "1")
        ref = e.snapshot_batch(batch)
    bad = [k for k in range(len(batch)) if got[k] != ref[k]]
    assert not bad, f"{len(bad)} documents differ between the tiers, first {bad[:5]}"
    assert sum(st == 0 for st, _ in got) >= len(batch) - 3


@pytest.mark.gpu
def test_gpu_snapshot_envelope():
    """A gap and a missing origin leave pending structs: yjs 13.5.16 answers with the structs themselves (its bytes,
    computed by the bundle: node -e ... Y.encodeStateAsUpdate(applyUpdate(new Doc, u))); an empty update is malformed
    (yjs throws)."""
    from hocuspocus_amd import Engine
    from hocuspocus_amd.engine import EMALFORMED
    with Engine(0, compat135=True) as e:
        gap = bytes([1, 1, 5, 3, 0x04, 1, 1, 0x74, 1, 0x61, 0])   # client 5 starts at clock 3: pending
        orphan = bytes([1, 1, 5, 0, 0x84, 9, 0, 1, 0x61, 0])   # origin (9, 0) is not in the update
        res = e.snapshot_batch([gap, orphan, b""])
        assert res[0] == (0, bytes.fromhex("0101050304010174016100"))
        assert res[1] == (0, bytes.fromhex("01010500840900016100"))
        assert res[2][0] == EMALFORMED


# ---------------------------------------------------------------------------------------- pending structs / delete set
# tests/golden/snapshot_pending_v135.json.gz: the generator's sessions with 1-3 of the log's updates lost
# (tools/snap_fixture.py 200:31:120:pending 120:32:200:textpending): applyUpdate leaves pending structs and / or a
# pending delete set, and encodeStateAsUpdate merges [state, pendingDs, pending structs] (Y@23300).
PFIX = os.path.join(ROOT, "tests", "golden", "snapshot_pending_v135.json.gz")


def pending_fixtures():
    d = json.load(gzip.open(PFIX, "rt"))
    return [(bytes.fromhex(u), bytes.fromhex(e)) for u, e in d["rows"]]


def test_pending_fixtures_present():
    rows = pending_fixtures()
    assert len(rows) == 320 and all(u and e for u, e in rows)


@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle are needed to regenerate")
def test_pending_fixtures_regenerate(tmp_path):
    """The committed vectors are what the generator's pending mode produces from the bundle (first sessions)."""
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "exp.bin")
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_corpus.js"), "30", "31", a, b, "120", "pending"], check=True, timeout=120)
    rows = pending_fixtures()[:30]
    assert read_in(a) == [u for u, _ in rows]
    assert [e for _, e in read_res(b)] == [e for _, e in rows]


def _resolve_pending(st, body, compat135):
    """A host-compiled kernel result: status 64 (snap::ST_PEND) carries PendHdr + [state, pendingDs, pending structs],
    which the engine merges with the merge kernels -- here the oracle's mergeUpdates does that step."""
    import oracle
    if st != 64:
        return st, body
    ln = struct.unpack_from("<IIII", body, 0)
    assert ln[3] == 0x444E4550
    parts, p = [], 16
    for k in range(3):
        parts.append(body[p:p + ln[k]])
        p += ln[k]
    return oracle.merge_updates(parts, compat135=compat135)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("mode", [1, 0])
def test_pending_kernel_code_on_host(tmp_path, mode):
    """The kernel's code host-compiled over the pending vectors: most documents come out pending (the dependency
    stack's rest and the delete set past the state), and merging their three updates gives yjs's bytes (13.5) / the
    client-descending delete sets (default)."""
    from golden import ds_to_desc
    exe = str(tmp_path / "snapdev")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "snapdev", "snapdev.cpp")], check=True, timeout=300)
    rows = pending_fixtures()
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_in(a, [u for u, _ in rows])
    subprocess.run([exe, a, b, str(mode)], check=True, timeout=120)
    got = read_res(b)
    assert sum(st == 64 for st, _ in got) >= 200
    exp = [(0, e) if mode else (0, bytes.fromhex(ds_to_desc(e.hex()))) for _, e in rows]
    res = [_resolve_pending(st, body, bool(mode)) for st, body in got]
    bad = [k for k in range(len(rows)) if res[k] != exp[k]]
    assert not bad, f"{len(bad)} documents differ, first {bad[:5]}"


# sub-documents (ContentDoc: Y.Doc values in a map and an array, overwritten and deleted ones among them), complete and
# with lost updates (tools/snap_fixture.py 160:61:120:subdoc 100:62:120:subpending)
SFIX = os.path.join(ROOT, "tests", "golden", "snapshot_subdoc_v135.json.gz")


def subdoc_fixtures():
    d = json.load(gzip.open(SFIX, "rt"))
    return [(bytes.fromhex(u), bytes.fromhex(e)) for u, e in d["rows"]]


def test_subdoc_fixtures_present():
    rows = subdoc_fixtures()
    assert len(rows) == 260 and all(u and e for u, e in rows)


@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle are needed to regenerate")
def test_subdoc_fixtures_regenerate(tmp_path):
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "exp.bin")
    subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_corpus.js"), "20", "61", a, b, "120", "subdoc"], check=True, timeout=120)
    rows = subdoc_fixtures()[:20]
    assert read_in(a) == [u for u, _ in rows]
    assert [e for _, e in read_res(b)] == [e for _, e in rows]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("mode", [1, 0])
def test_subdoc_kernel_code_on_host(tmp_path, mode):
    """Sub-documents through the kernel's code host-compiled: ContentDoc items integrate, split never (one clock), and
    are garbage-collected to ContentDeleted when deleted; canonical options are written as read."""
    from golden import ds_to_desc
    exe = str(tmp_path / "snapdev")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "snapdev", "snapdev.cpp")], check=True, timeout=300)
    rows = subdoc_fixtures()
    a, b = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_in(a, [u for u, _ in rows])
    subprocess.run([exe, a, b, str(mode)], check=True, timeout=120)
    exp = [(0, e) if mode else (0, bytes.fromhex(ds_to_desc(e.hex()))) for _, e in rows]
    res = [_resolve_pending(st, body, bool(mode)) for st, body in read_res(b)]
    bad = [k for k in range(len(rows)) if res[k] != exp[k]]
    assert not bad, f"{len(bad)} documents differ, first {bad[:5]}"


@pytest.mark.gpu
def test_gpu_snapshot_subdocs_vs_yjs(eng135):
    rows = subdoc_fixtures()
    res = eng135.snapshot_batch([u for u, _ in rows])
    bad = [k for k, ((_, e), r) in enumerate(zip(rows, res)) if r != (0, e)]
    assert not bad, f"{len(bad)} documents differ from yjs, first {bad[:5]}: {res[bad[0]]}"


@pytest.mark.gpu
def test_gpu_snapshot_pending_vs_yjs_fixtures(eng135):
    """On the GPU (13.5): the pending documents' three updates merged by the merge kernels give yjs's bytes."""
    rows = pending_fixtures()
    s0 = eng135.stats()
    res = eng135.snapshot_batch([u for u, _ in rows])
    bad = [k for k, ((_, e), r) in enumerate(zip(rows, res)) if r != (0, e)]
    assert not bad, f"{len(bad)} documents differ from yjs, first {bad[:5]}: {res[bad[0]]}"
    assert eng135.stats().docs_pending - s0.docs_pending >= 200


@pytest.mark.gpu
def test_gpu_snapshot_pending_default_mode():
    """The same in the 13.6 default mode, against client-descending delete sets; mixed with complete documents."""
    from golden import ds_to_desc
    from hocuspocus_amd import Engine
    rows = pending_fixtures() + fixtures()[:100]
    with Engine(0) as e:
        res = e.snapshot_batch([u for u, _ in rows])
    exp = [(0, bytes.fromhex(ds_to_desc(x.hex()))) for _, x in rows]
    bad = [k for k in range(len(rows)) if res[k] != exp[k]]
    assert not bad, f"{len(bad)} documents differ, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle (image) needed for live sessions")
def test_gpu_snapshot_pending_live_yjs(eng135, tmp_path):
    """Fresh pending sessions generated on this box by yjs (both generator shapes, longer sessions)."""
    batch, exp = [], []
    for seed, ops, mode in ((41, 200, "pending"), (42, 400, "textpending")):
        a, b = str(tmp_path / f"in{seed}.bin"), str(tmp_path / f"exp{seed}.bin")
        subprocess.run([NODE, os.path.join(ROOT, "tools", "snap_corpus.js"), "150", str(seed), a, b, str(ops), mode], check=True, timeout=240)
        batch += read_in(a)
        exp += [e for _, e in read_res(b)]
    res = eng135.snapshot_batch(batch)
    bad = [k for k in range(len(batch)) if res[k] != (0, exp[k])]
    assert not bad, f"{len(bad)} documents differ, first {bad[:5]}"


# ---------------------------------------------------------------------------------------- read-only SyncStep2
CFIX = os.path.join(ROOT, "tests", "golden", "contains_v135.json.gz")


def contains_fixtures():
    d = json.load(gzip.open(CFIX, "rt"))
    states = [bytes.fromhex(s) for s in d["states"]]
    return [(states[i], bytes.fromhex(u), bool(e)) for i, u, e in d["rows"]]


def test_contains_fixtures_present():
    rows = contains_fixtures()
    assert len(rows) > 300 and 0 < sum(e for _, _, e in rows) < len(rows)


@pytest.mark.gpu
def test_gpu_contains_vs_yjs_fixtures():
    """Y.snapshotContainsUpdate(Y.snapshot(doc), update) (MessageReceiver.ts:156-179) on the GPU."""
    from hocuspocus_amd import Engine
    rows = contains_fixtures()
    with Engine(0) as e:
        res = e.contains_batch([s for s, _, _ in rows], [u for _, u, _ in rows])
    assert res == [(0, x) for _, _, x in rows]


@pytest.mark.gpu
@pytest.mark.skipif(not (NODE and BUNDLE), reason="node + the yjs bundle (image) needed")
def test_gpu_contains_vs_live_yjs(tmp_path):
    from hocuspocus_amd import Engine
    a, b, c = str(tmp_path / "st.bin"), str(tmp_path / "up.bin"), str(tmp_path / "ex.bin")
    subprocess.run([NODE, os.path.join(ROOT, "tools", "contains_corpus.js"), "150", "77", a, b, c], check=True, timeout=240)
    st, up, ex = read_in(a), read_in(b), list(open(c, "rb").read())
    with Engine(0) as e:
        res = e.contains_batch(st, up)
        # the GPU's own normalized states answer the same
        snaps = e.snapshot_batch(st)
        res2 = e.contains_batch([s for _, s in snaps], up)
    assert res == [(0, bool(x)) for x in ex]
    assert res2 == res


# pending states (tools/snap_fixture.py --contains 120 51 pending): the stored state is the merge of a history with
# lost updates -- its document keeps pending structs / a pending delete set, and Y.snapshot(doc) sees the store alone
PCFIX = os.path.join(ROOT, "tests", "golden", "contains_pending_v135.json.gz")


def contains_pending_fixtures():
    d = json.load(gzip.open(PCFIX, "rt"))
    states = [bytes.fromhex(s) for s in d["states"]]
    return [(states[i], bytes.fromhex(u), bool(e)) for i, u, e in d["rows"]]


def test_contains_pending_fixtures_present():
    rows = contains_pending_fixtures()
    assert len(rows) > 300 and 0 < sum(e for _, _, e in rows) < len(rows)


@pytest.mark.gpu
def test_gpu_contains_pending_states_vs_yjs():
    """Read-only SyncStep2 against states that leave pending parts: the containment runs on the state's Y.snapshot
    view (its integrated part), on the GPU, with no host yjs; in both modes, mixed with complete states."""
    from hocuspocus_amd import Engine
    rows = contains_pending_fixtures() + contains_fixtures()[:100]
    for compat in (True, False):
        with Engine(0, compat135=compat) as e:
            res = e.contains_batch([s for s, _, _ in rows], [u for _, u, _ in rows])
        assert res == [(0, x) for _, _, x in rows]
