"""N>1 path on CPU: world_size-2 gloo processes partition documents by name hash,
merge their shards (CPU oracle stands in for the per-GPU engine here: no GPU in
this container) and gather node totals -- the same partition + stats-gather code
bench.py and a multi-GPU deployment use."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    import oracle
    from hocuspocus_amd.shard import gather_stats, partition
    from tools import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    arena, upd_off, doc_upd = synth.text_updates(64, 30, seed=77, del_pct=10)
    ups = synth.split(arena, upd_off)
    names = [f"doc-{i}" for i in range(64)]
    mine = partition(names, world)[rank]
    b_in = b_out = 0
    digest = {}
    for i in mine:
        us = ups[doc_upd[i]:doc_upd[i + 1]]
        st, out = oracle.merge_updates(us)
        assert st == 0
        b_in += sum(map(len, us))
        b_out += len(out)
        digest[names[i]] = out.hex()
    tot = gather_stats({"docs": len(mine), "bytes_in": b_in, "bytes_out": b_out, "kernel_ms": 1.0 + rank}, dist)
    q.put((rank, tot, digest))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300) if hasattr(pytest.mark, "timeout") else (lambda f: f)
def test_two_rank_gloo_partition_and_stats():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    t0, t1 = res[0][1], res[1][1]
    assert t0 == t1 and t0["ranks"] == 2 and t0["docs"] == 64 and t0["kernel_ms"] == 2.0
    d0, d1 = res[0][2], res[1][2]
    assert not (set(d0) & set(d1)) and len(d0) + len(d1) == 64     # disjoint shards, all documents
    # single-process reference totals
    import oracle
    from tools import synth
    arena, upd_off, doc_upd = synth.text_updates(64, 30, seed=77, del_pct=10)
    ups = synth.split(arena, upd_off)
    ref_out = sum(len(oracle.merge_updates(ups[doc_upd[i]:doc_upd[i + 1]])[1]) for i in range(64))
    assert t0["bytes_out"] == ref_out and t0["bytes_in"] == len(arena)


def test_shard_of_is_stable():
    from hocuspocus_amd.shard import fnv1a64, shard_of
    assert fnv1a64(b"") == 0xCBF29CE484222325
    assert fnv1a64(b"a") == 0xAF63DC4C8601EC8C  # FNV-1a 64 test vector
    assert all(0 <= shard_of(f"d{i}", 8) < 8 for i in range(100))


def test_sharded_engine_routes_and_reassembles():
    # single-process multi-GPU form: documents routed by fnv1a64(name) mod N, results in caller order
    # (the CPU oracle stands in for the per-device engine here)
    import oracle
    from hocuspocus_amd.shard import ShardedEngine, shard_of
    from tools import synth

    class OracleEngine:
        def __init__(self):
            self.docs = []

        def merge_updates_batch(self, docs):
            self.docs.append(len(docs))
            return [oracle.merge_updates(us) for us in docs]

    engines = [OracleEngine() for _ in range(3)]
    se = ShardedEngine(engines=engines)
    arena, upd_off, doc_upd = synth.text_updates(40, 12, seed=5)
    ups = synth.split(arena, upd_off)
    docs = [ups[doc_upd[d]:doc_upd[d + 1]] for d in range(40)]
    names = [f"room/{d}" for d in range(40)]
    res = se.merge_updates_batch(names, docs)
    assert res == [oracle.merge_updates(us) for us in docs]
    counts = [sum(1 for n in names if shard_of(n, 3) == k) for k in range(3)]
    assert [sum(e.docs) for e in engines] == counts and all(len(e.docs) <= 1 for e in engines)
    se.close()
