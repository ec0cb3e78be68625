"""Document sharding across GPUs.

Documents are independent, so a node's batch is partitioned by
``fnv1a64(utf8(documentName)) mod N`` with no cross-GPU exchange of update
data.  The only collective is the optional node-wide stats gather
(``gather_stats``): a fixed-size vector per rank over ``torch.distributed``
(RCCL on GPUs, gloo on CPU).
"""
from __future__ import annotations

FNV_OFFSET = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3
MASK64 = (1 << 64) - 1

STAT_FIELDS = ("docs", "updates", "bytes_in", "bytes_out", "docs_seq", "kernel_ms")


def fnv1a64(data: bytes) -> int:
    h = FNV_OFFSET
    for b in data:
        h ^= b
        h = (h * FNV_PRIME) & MASK64
    return h


def shard_of(document_name: str, n_shards: int) -> int:
    """GPU index that owns a document (stable across processes and restarts)."""
    return fnv1a64(document_name.encode("utf-8")) % n_shards


def partition(document_names, n_shards: int):
    """Indices of the documents owned by each shard, preserving order."""
    parts = [[] for _ in range(n_shards)]
    for i, name in enumerate(document_names):
        parts[shard_of(name, n_shards)].append(i)
    return parts


class ShardedEngine:
    """One process driving several GPUs of a node: one Engine (context + stream) per device,
    documents routed by ``shard_of(name, N)``; a batch is split by shard, the shards run
    concurrently (the C ABI releases the GIL for the whole call) and results come back in
    caller order.  Same batch API as :class:`hocuspocus_amd.engine.Engine` plus document names
    (mirror of ``GpuEnginePool`` in packages/extension-gpu-merge/src/engine.js)."""

    def __init__(self, devices=(0,), engines=None, **engine_kw):
        if engines is None:
            from .engine import Engine
            engines = [Engine(d, **engine_kw) for d in devices]
        self.engines = list(engines)
        from concurrent.futures import ThreadPoolExecutor
        self._pool = ThreadPoolExecutor(max_workers=len(self.engines))

    def _run(self, names, cols, call):
        parts = partition(names, len(self.engines))
        futs = {k: self._pool.submit(call, self.engines[k], *[[c[i] for i in idx] for c in cols])
                for k, idx in enumerate(parts) if idx}
        out = [None] * len(names)
        for k, f in futs.items():
            for i, r in zip(parts[k], f.result()):
                out[i] = r
        return out

    def merge_updates_batch(self, names, docs):
        return self._run(names, [docs], lambda e, d: e.merge_updates_batch(d))

    def diff_update_batch(self, names, updates, svs):
        return self._run(names, [updates, svs], lambda e, u, s: e.diff_update_batch(u, s))

    def encode_state_vector_from_update_batch(self, names, updates):
        return self._run(names, [updates], lambda e, u: e.encode_state_vector_from_update_batch(u))

    def close(self):
        self._pool.shutdown()
        for e in self.engines:
            if hasattr(e, "close"):
                e.close()


def gather_stats(stats: dict, dist=None, device=None):
    """All-gathers one fixed-size stats vector per rank and returns the node totals.
    kernel_ms is reduced with max (ranks run concurrently), everything else summed."""
    import torch
    vec = torch.tensor([float(stats.get(k, 0.0)) for k in STAT_FIELDS], dtype=torch.float64, device=device)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        rows = [vec]
    else:
        rows = [torch.empty_like(vec) for _ in range(dist.get_world_size())]
        dist.all_gather(rows, vec)
    stacked = torch.stack(rows).cpu()
    out = {k: float(stacked[:, i].sum()) for i, k in enumerate(STAT_FIELDS)}
    out["kernel_ms"] = float(stacked[:, STAT_FIELDS.index("kernel_ms")].max())
    out["ranks"] = len(rows)
    return out
