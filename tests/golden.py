"""Loader for the committed golden fixtures (tests/golden/*).

yjs13516_vectors.jsonl.gz -- made by tests/golden/gen/gen_fixtures.js from
yjs 13.5.16 (the copy JupyterLab bundles in the build image); see SURVEY.md §8c.
Each case: op in {merge, diff, sv}, hex inputs, hex `out` (None when yjs threw)
and `err` (yjs's exception text).
"""
import gzip
import json
import os

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# yjs throws on these; any engine error status is an acceptable equivalent.
THROW_STATUSES = {1, 2, 4, 5}  # EMALFORMED, ERANGE, ESURROGATE, EDEPTH
# Edge-family notes whose content yjs re-encodes; the
# engine may refuse them with ENONCANON instead of normalising.
NONCANON_NOTES = ("any ", "json ", "embed non-canonical", "format non-canonical", "doc {gc:true}")


def load_yjs_vectors():
    with gzip.open(os.path.join(HERE, "yjs13516_vectors.jsonl.gz")) as f:
        lines = f.read().decode().splitlines()
    header = json.loads(lines[0])
    cases = [json.loads(l) for l in lines[1:]]
    assert header["count"] == len(cases)
    return header, cases


def load_v8_sort_vectors():
    with gzip.open(os.path.join(HERE, "v8_timsort_vectors.json.gz")) as f:
        return json.loads(f.read())


def case_inputs(c):
    if c["op"] == "merge":
        return [bytes.fromhex(x) for x in c["in"]]
    if c["op"] == "diff":
        return bytes.fromhex(c["update"]), bytes.fromhex(c["sv"])
    return bytes.fromhex(c["update"])


def check_result(c, status, out):
    """Returns None if (status, out) is an acceptable answer for golden case c, else a reason."""
    exp = c["out"]
    if exp is None:
        return None if status in THROW_STATUSES else f"yjs threw ({c['err']}) but got status {status}"
    if status == 0:
        return None if out.hex() == exp else f"bytes differ:\n exp {exp}\n got {out.hex()}"
    if status == 3 and c["family"] == "edge" and (c.get("note") or "").startswith(NONCANON_NOTES):
        return None
    return f"status {status} but yjs returned {exp}"


def ds_to_desc(update_hex):
    """Rewrites an output's delete set into client-descending order (yjs 13.6.x writeDeleteSet)."""
    from v1util import ds_offset, encode_ds, read_ds
    b = bytes.fromhex(update_hex)
    p = ds_offset(b)
    ds, _ = read_ds(b, p)
    return (b[:p] + encode_ds(sorted(ds, key=lambda e: -e[0]))).hex()
