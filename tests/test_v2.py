"""Update-V2 codec: yjs mergeUpdatesV2 / diffUpdateV2 / encodeStateVectorFromUpdateV2 and
yjs 13.6's convertUpdateFormatV1ToV2 / V2ToV1.

CPU tests pin the oracle (oracle/yjs_oracle_v2.c) against tests/golden/yjs13516_v2_vectors.jsonl.gz, made by
tests/golden/gen/gen_v2.js from the yjs 13.5.16 bundle in the build image.  GPU tests (-m gpu) run the same
vectors through the C ABI (ygm_*_v2) and compare with yjs's bytes, then larger synthetic V2 corpora against
the oracle.
"""
import gzip
import json
import os

import pytest

import oracle

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
THROW = {1, 2, 4, 5}


def load_v2_vectors():
    with gzip.open(os.path.join(HERE, "yjs13516_v2_vectors.jsonl.gz")) as f:
        lines = f.read().decode().splitlines()
    header = json.loads(lines[0])
    cases = [json.loads(l) for l in lines[1:]]
    assert header["count"] == len(cases)
    return cases


def check(c, st, out):
    """(status, bytes) acceptable for golden case c?  Inputs derived from malformed bytes ('-bad' families)
    may be refused (ENONCANON: e.g. a string slice that splits a surrogate pair has no V1 form)."""
    exp = c["out"]
    bad = c["family"].endswith("-bad")
    if exp is None:
        return st in THROW or (st == 3 and bad)
    return (st == 0 and out is not None and out.hex() == exp) or (st == 3 and bad)


def run_oracle(c, compat=True):
    if c["op"] == "merge_v2":
        return oracle.merge_updates_v2([bytes.fromhex(x) for x in c["in"]], compat135=compat)
    if c["op"] == "diff_v2":
        return oracle.diff_update_v2(bytes.fromhex(c["update"]), bytes.fromhex(c["sv"]), compat135=compat)
    return oracle.encode_state_vector_from_update_v2(bytes.fromhex(c["update"]), compat135=compat)


def test_oracle_v2_vs_yjs():
    cases = load_v2_vectors()
    n = {"merge_v2": 0, "diff_v2": 0, "sv_v2": 0}
    for c in cases:
        if c["op"] == "conv":
            continue
        st, out = run_oracle(c)
        assert check(c, st, out), (c, st, out and out.hex())
        n[c["op"]] += 1
    assert min(n.values()) > 500


def test_oracle_convert_vs_yjs_pairs():
    exact = refused = 0
    for c in load_v2_vectors():
        if c["op"] != "conv":
            continue
        v1, v2 = bytes.fromhex(c["v1"]), bytes.fromhex(c["v2"])
        assert oracle.convert_update_format_v1_to_v2(v1, compat135=True) == (0, v2), c
        st, out = oracle.convert_update_format_v2_to_v1(v2, compat135=True)
        if st == 3:   # a float (or undefined / binary) inside an embed / format value: refused
            refused += 1
        else:
            assert (st, out) == (0, v1), c
            exact += 1
    assert exact > 500 and refused < exact


def test_oracle_v2_default_mode_matches_compat_up_to_ds_order():
    """13.6 default differs from 13.5 only in delete-set client order: equal bytes whenever the delete set
    has at most one client."""
    diff = same = 0
    for c in load_v2_vectors():
        if c["op"] != "merge_v2" or c["out"] is None or c["family"].endswith("-bad"):
            continue   # (malformed inputs: lib0 0.2.42 / 0.2.104 read truncated strings differently)
        a = run_oracle(c, True)
        b = run_oracle(c, False)
        assert (a[0] == 0) == (b[0] == 0) or a[0] == 3 or b[0] == 3
        if a[0] == 0 and b[0] == 0:
            if a[1] == b[1]:
                same += 1
            else:
                diff += 1
    assert same > 100


def test_v2_empty_merge_is_the_empty_v2_update():
    st, out = oracle.merge_updates_v2([], compat135=True)
    assert st == 0 and out == bytes([0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0])
    # single input: returned as-is, not parsed (yjs Y@39011)
    assert oracle.merge_updates_v2([b"\xff\xff"]) == (0, b"\xff\xff")


# ------------------------------------------------------------------ GPU (through the C ABI)
@pytest.fixture(scope="module")
def eng135():
    from hocuspocus_amd import Engine
    e = Engine(0, compat135=True)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng():
    from hocuspocus_amd import Engine
    e = Engine(0)
    yield e
    e.close()


def gpu_batch(e, op, cases):
    if op == "merge_v2":
        return e.merge_updates_v2_batch([[bytes.fromhex(x) for x in c["in"]] for c in cases])
    if op == "diff_v2":
        return e.diff_update_v2_batch([bytes.fromhex(c["update"]) for c in cases], [bytes.fromhex(c["sv"]) for c in cases])
    return e.encode_state_vector_from_update_v2_batch([bytes.fromhex(c["update"]) for c in cases])


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["merge_v2", "diff_v2", "sv_v2"])
def test_gpu_v2_vs_yjs(eng135, op):
    cases = [c for c in load_v2_vectors() if c["op"] == op]
    res = gpu_batch(eng135, op, cases)
    bad = [(c, st, out and out.hex()) for c, (st, out) in zip(cases, res) if not check(c, st, out)]
    assert not bad, (len(bad), bad[:3])


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["merge_v2", "diff_v2", "sv_v2"])
def test_gpu_v2_default_mode_vs_oracle(eng, op):
    cases = [c for c in load_v2_vectors() if c["op"] == op]
    res = gpu_batch(eng, op, cases)
    for c, (st, out) in zip(cases, res):
        so, oo = run_oracle(c, compat=False)
        if so in THROW:
            assert st in THROW or (st == 3 and c["family"].endswith("-bad")), (c, st)
        else:
            assert (st, out) == (so, oo) or (st == 3 and c["family"].endswith("-bad")), (c, st, so)


@pytest.mark.gpu
def test_gpu_convert_vs_yjs_pairs(eng135):
    pairs = [c for c in load_v2_vectors() if c["op"] == "conv"]
    v1s = [bytes.fromhex(c["v1"]) for c in pairs]
    v2s = [bytes.fromhex(c["v2"]) for c in pairs]
    for c, v2, (st, out) in zip(pairs, v2s, eng135.convert_update_format_v1_to_v2_batch(v1s)):
        assert (st, out) == (0, v2), c
    refused = 0
    for c, v1, (st, out) in zip(pairs, v1s, eng135.convert_update_format_v2_to_v1_batch(v2s)):
        if st == 3:
            refused += 1
            assert oracle.convert_update_format_v2_to_v1(bytes.fromhex(c["v2"]), compat135=True)[0] == 3, c
        else:
            assert (st, out) == (0, v1), c
    assert refused < len(pairs) // 3


@pytest.mark.gpu
def test_gpu_v2_synthetic_logs_vs_oracle(eng):
    """C2-shaped logs (with deletions, 1-4 clients) converted to V2: merged on the GPU, then diffed and state-vectored,
    each against the oracle; plus the V2 -> V1 -> V2 conversion round trip of the merged states."""
    from tools import synth
    n_docs = 1500
    arena, upd_off, doc_upd = synth.text_updates(n_docs, 30, seed=23, del_pct=20)
    ups = synth.split(arena, upd_off)
    v1docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(n_docs)]
    v2docs = [[oracle.convert_update_format_v1_to_v2(u)[1] for u in us] for us in v1docs]
    got = eng.merge_updates_v2_batch(v2docs)
    merged = []
    for d, us in enumerate(v2docs):
        exp = oracle.merge_updates_v2(us)
        assert got[d] == exp, d
        merged.append(exp[1])
    svs = eng.encode_state_vector_from_update_v2_batch(merged)
    half = []
    for d, m in enumerate(merged):
        assert svs[d] == oracle.encode_state_vector_from_update_v2(m), d
        half.append(oracle.encode_state_vector_from_update_v2(oracle.merge_updates_v2(v2docs[d][: len(v2docs[d]) // 2])[1])[1])
    diffs = eng.diff_update_v2_batch(merged, half)
    for d, m in enumerate(merged):
        assert diffs[d] == oracle.diff_update_v2(m, half[d]), d
    back = eng.convert_update_format_v2_to_v1_batch(merged)
    for d, m in enumerate(merged):
        assert back[d] == oracle.convert_update_format_v2_to_v1(m), d
    again = eng.convert_update_format_v1_to_v2_batch([b for _, b in back])
    assert again == [(0, m) for m in merged]
