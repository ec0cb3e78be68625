"""CPU check of the tile-edge documents the GPU parity test feeds k_merge_big: every one is a valid
input yjs merges (oracle status 0), over the 16 KB that routes it to the large-document tier, and
holds what the tiled walk hands to global memory (a string longer than a tile's 2 KB overlap,
ContentJSON over the 8 entries the speculative parse takes, more than 256 client blocks)."""
import oracle
from tile_docs import tile_edge_docs


def test_tile_edge_docs_are_valid_large_inputs():
    docs = tile_edge_docs(5)
    assert len(docs) == 6
    for us in docs:
        assert len(us[0]) > 16384
        st, out = oracle.merge_updates(us)
        assert st == 0 and len(out) >= len(us[0])
    snap = docs[-1][0]
    assert snap.count(b"\x82") > 0          # ContentJSON info bytes present
    assert max(len(us[0]) for us in docs) > 1_000_000


def test_ds_splice_docs_are_valid_large_inputs():
    from tile_docs import ds_splice_docs
    for seed in (11, 12, 13):
        docs = ds_splice_docs(seed)
        for us in docs:
            assert len(us[0]) > 16384
            assert oracle.merge_updates(us)[0] == 0
