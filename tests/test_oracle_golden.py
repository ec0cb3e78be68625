"""The CPU oracle (oracle/yjs_oracle.c) pinned against yjs's own outputs.

Every vector in tests/golden/yjs13516_vectors.jsonl.gz was produced by running
yjs 13.5.16 (SURVEY.md §8c secondary oracle); the oracle runs in its
13.5.16-compat mode for these.  The V8 TimSort vectors pin the decoder re-sort
of mergeUpdates (Y@39011) under its inconsistent comparator.
"""
import collections

import pytest

import oracle
from golden import case_inputs, check_result, load_v8_sort_vectors, load_yjs_vectors

HEADER, CASES = load_yjs_vectors()


def run_oracle(c, compat135=True):
    if c["op"] == "merge":
        return oracle.merge_updates(case_inputs(c), compat135=compat135)
    if c["op"] == "diff":
        u, sv = case_inputs(c)
        return oracle.diff_update(u, sv, compat135=compat135)
    return oracle.encode_state_vector_from_update(case_inputs(c), compat135=compat135)


def test_fixture_header():
    assert HEADER["oracle"] == "yjs13.5.16/lib0-0.2.42"
    assert len(CASES) > 8000
    ops = collections.Counter(c["op"] for c in CASES)
    assert ops["merge"] > 2000 and ops["diff"] > 2000 and ops["sv"] > 2000


@pytest.mark.parametrize("family", sorted({c["family"].split("-")[0] for c in CASES}))
def test_oracle_matches_yjs(family):
    fails = []
    for c in CASES:
        if c["family"].split("-")[0] != family:
            continue
        st, out = run_oracle(c)
        why = check_result(c, st, out)
        if why:
            fails.append((c["id"], c.get("note"), why))
    assert not fails, f"{len(fails)} mismatches, first: {fails[:3]}"


def test_noncanonical_refusals_are_real():
    # every ENONCANON refusal must be a case where yjs really re-encoded the content
    n = 0
    for c in CASES:
        if c["op"] != "merge" or c["out"] is None:
            continue
        st, _ = run_oracle(c)
        if st == 3:
            n += 1
            assert c["out"] != c["in"][0], c
    assert n > 10


def test_v8_timsort_emulation():
    d = load_v8_sort_vectors()
    for c in d["cases"]:
        n = c["n"]
        key, kind = c["key"], c["kind"]
        T = [0] * (n * n)
        for a in range(n):
            for b in range(n):
                if key[a] != key[b]:
                    T[a * n + b] = -1 if key[a] < key[b] else 1
                else:
                    T[a * n + b] = 0 if kind[a] == kind[b] else -1
        for a, b, v in c["noise"]:
            T[a * n + b] = v
        out, calls = oracle.v8_sort_table(c["input"], T)
        assert out == c["out"] and calls == c["calls"], (n, calls, c["calls"])


def test_default_mode_13_6_ds_order():
    # 13.6.x writes delete-set clients in descending order
    st, out = oracle.merge_updates([bytes.fromhex("00020201000109010001"), bytes.fromhex("0000")])
    assert st == 0 and out.hex() == "00020901000102010001"
    st, out = oracle.merge_updates([bytes.fromhex("00020201000109010001"), bytes.fromhex("0000")], compat135=True)
    assert out.hex() == "00020201000109010001"


def test_default_mode_lone_surrogate_written_as_fffd():
    u = bytes.fromhex("01010500040101740661f09f98806200")  # 'a😀b', client 5
    st, _ = oracle.diff_update(u, bytes.fromhex("010502"), compat135=True)
    assert st == 4  # 13.5.16 throws (URI malformed)
    st, out = oracle.diff_update(u, bytes.fromhex("010502"))
    assert st == 0 and out.hex() == "01010502840501" + "04efbfbd62" + "00"


# lib0 0.2.42 writes negative integer floats below -2^31 as varInt (no abs, L0@8319);
# 0.2.104 keeps them f64: the 13.5.16 vector is not the 13.6.26 answer.
VERSION_SENSITIVE_NOTES = {"any 7bc1e0000000200000"}


def test_default_mode_equals_13_5_up_to_ds_order():
    # 13.6.26 semantics = the 13.5.16 vectors with client-descending delete sets,
    # except lone-surrogate writes (throw in 13.5.16, U+FFFD in 13.6.x: unpinned)
    from golden import ds_to_desc
    n = 0
    for c in CASES:
        if c["op"] == "sv" or c["out"] is None:
            continue
        st, out = run_oracle(c, compat135=False)
        if st == 3 and check_result(c, 3, None) is None:
            continue
        if (c.get("note") or "") in VERSION_SENSITIVE_NOTES:
            continue
        if c["op"] == "merge" and len(c["in"]) == 1:
            assert out.hex() == c["out"]
            continue
        assert st == 0, (c["id"], st)
        assert out.hex() == ds_to_desc(c["out"]), c["id"]
        n += 1
    assert n > 4000
