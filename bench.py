"""Benchmark: batched Y.mergeUpdates on MI355X (BASELINE.json metric, config C2).

    python bench.py [--gpus N] [--steps K] [--warmup W]

One step = one batched mergeUpdates over the whole per-GPU workload (10 000
documents x 200 single-character Y.Text insert updates from 1-4 clients,
SURVEY.md §8d config C2, BASELINE.json configs[1]) with the inputs already
resident in HBM: ``ygm_merge_v1_device_async`` = the counter reset and the lean
kernel launch, each document written into its own output slot.  Steps are enqueued
back to back on one stream; the last one is completed by ``ygm_merge_v1_device_finish``
(fault check, payload).  Every C2 document is finished by the lean kernel -- asserted
on the warmup (identical inputs every step) and on the timed run -- so no step needs
the host-driven wave / workgroup / sequential tiers.  For N > 1 the
driver starts one process per GPU (torchrun); every rank merges its own shard
of documents (documents are independent, partitioned by name hash, weak
scaling) and the time is the max over ranks.  RCCL carries only the timing
reduction / stats gather, never data.

Algorithmic bytes: merge = sum(|inputs|) + |output| per document.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
N_DOCS, N_UPDATES = 10000, 200
PMC_PROFILE = "r01_big_v4/pmc_hbm.json"  # latest committed PMC summary of the bench kernel


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=N_DOCS)
    ap.add_argument("--updates", type=int, default=N_UPDATES)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--big", choices=["c3", "c5"], default=None,
                    help="instead of the C2 line: one C3 / C5 large-document batch on the GPU next to the CPU oracle "
                         "over the same documents (reported beside the headline, never as it)")
    ap.add_argument("--big-docs", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(arena, upd_off, doc_upd, budget_s):
    """The CPU oracle (oracle/yjs_oracle.c: a literal C restatement of yjs mergeUpdates,
    "port") on a bounded sample of the same workload, one pthread per host core."""
    import oracle
    n_docs = len(doc_upd) - 1
    cores = min(16, os.cpu_count() or 1)

    def run(n, threads):
        sub_upd = doc_upd[:n + 1]
        t0 = time.perf_counter()
        st, algo = oracle.merge_batch(arena, upd_off, sub_upd, threads)
        return time.perf_counter() - t0, algo, st

    # calibrate on one thread, then size the sample for ~budget_s of all-core work
    n0 = min(n_docs, 200)
    dt0, _, _ = run(n0, 1)
    per_doc = dt0 / n0
    sample = int(min(n_docs, max(n0, budget_s * cores / per_doc)))
    # repeat passes over the sample until ~budget_s of all-core CPU work has been timed
    dt, algo, reps = 0.0, 0, 0
    while reps == 0 or dt * cores < budget_s:
        t, a, st = run(sample, cores)
        assert (st == 0).all()
        dt += t; algo += a; reps += 1
    return {"value": round(algo / dt / 1e6, 3), "unit": "MB/s", "cores": cores, "kind": "port",
            "docs_per_s": round(sample * reps / dt, 1),
            "sample": f"{reps} pass(es) over {sample} of the {n_docs} C2 documents through oracle/yjs_oracle.c "
                      f"yo_merge_batch (literal C restatement of yjs mergeUpdates incl. its V8-TimSort decoder "
                      f"loop), {cores} pthreads, {dt:.2f} s wall"}


def big_line(args):
    """C3 / C5 ([snapshot, ...log] large documents): the whole batch merged on cuda:0
    (device-resident inputs, host-driven tier cascade, kernel time from the engine's HIP events) and
    by the CPU oracle on all host threads over the same documents."""
    import torch
    import oracle
    from hocuspocus_amd import Engine
    from tools import synth
    xml = args.big == "c5"
    n = args.big_docs or (20 if xml else 2000)
    if xml:
        arena, upd_off, doc_upd = synth.big_docs(n, 1_000_000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
    else:
        arena, upd_off, doc_upd = synth.big_docs(n, 1_000_000, 1024, max_clients=64, max_k=200, seed=8)
    dev = torch.device("cuda", 0)
    da = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).to(dev)
    do = torch.from_numpy(upd_off.view(np.int64)).to(dev)
    dd = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
    e = Engine(0)
    for _ in range(2):   # the second run is timed (scratch already grown)
        s0 = e.stats()
        r = e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), n)
        s1 = e.stats()
    ms = s1.kernel_ms - s0.kernel_ms
    algo = len(arena) + r.payload_bytes
    cores = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    st, calgo = oracle.merge_batch(arena, upd_off, doc_upd, cores)
    cdt = time.perf_counter() - t0
    assert (st == 0).all()
    sizes = np.diff(upd_off[doc_upd].astype(np.int64))
    print(json.dumps({"config": args.big.upper(), "op": "merge", "docs": n, "bytes_in": len(arena), "largest_doc": int(sizes.max()),
                      "gpu_ms": round(ms, 3), "gpu_MBps": round(algo / ms / 1e3, 1), "gpu_docs_per_s": round(n / ms * 1e3),
                      "docs_big_tier": s1.docs_big - s0.docs_big, "docs_seq_tier": s1.docs_seq - s0.docs_seq,
                      "cpu_baseline": {"ms": round(cdt * 1e3, 3), "MBps": round(calgo / cdt / 1e6, 1), "cores": cores, "kind": "port",
                                       "sample": "all documents of the batch through oracle/yjs_oracle.c yo_merge_batch, one pass"}}),
          flush=True)


def main():
    args = parse()
    if args.big:
        return big_line(args)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from hocuspocus_amd import Engine
    from tools import synth

    # ---- this rank's shard: documents whose name hash maps to this rank (seeded per rank)
    arena, upd_off, doc_upd = synth.text_updates(args.docs, args.updates, seed=1000 + rank)
    n_upd = int(doc_upd[-1])
    dev = torch.device("cuda", local)
    d_arena = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).to(dev)
    d_off = torch.from_numpy(upd_off.view(np.int64)).to(dev)
    d_doc = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(local)

    def step():
        # one batched merge of the shard, enqueued on the stream (counter reset + lean kernel);
        # back-to-back steps pipeline.  Every document of this workload is finished by the lean
        # kernel (asserted on the warmup below: the inputs are identical in every step), so each
        # enqueued step is a complete merge without the host-driven tiers of finish().
        eng.merge_device_async(d_arena.data_ptr(), len(arena), d_off.data_ptr(), d_doc.data_ptr(), n_upd, args.docs,
                               stream.cuda_stream)

    w0 = eng.stats()
    for _ in range(max(args.warmup, 1)):
        step()
        eng.merge_device_finish()
    torch.cuda.synchronize()
    s0 = eng.stats()
    assert s0.docs_lean - w0.docs_lean == args.docs * max(args.warmup, 1), "not every document takes the lean kernel"
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    # finish the last step: fault check, payload (and no deferred document, as on the warmup)
    r = eng.merge_device_finish()
    s1 = eng.stats()
    assert s1.docs_lean - s0.docs_lean == args.docs, "a timed step deferred documents to the host-driven tiers"

    out_bytes = int(r.payload_bytes)                 # sum of the merged outputs' lengths
    algo_bytes = len(arena) + out_bytes              # per step, this rank
    # HIP events on the launch stream: one span over the timed back-to-back lean launches
    kernel_ms = (s1.lean_ms - s0.lean_ms) / max(s1.lean_launches - s0.lean_launches, 1)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)   # the job's time = the slowest rank
    dt = float(t.item())
    # node-wide stats all-gather (the only other collective; no update data crosses GPUs)
    from hocuspocus_amd.shard import gather_stats
    node = gather_stats({"docs": args.docs, "updates": n_upd, "bytes_in": len(arena), "bytes_out": out_bytes,
                         "docs_seq": s1.docs_seq - s0.docs_seq, "kernel_ms": kernel_ms}, dist, dev)
    all_bytes, all_docs = node["bytes_in"] + node["bytes_out"], node["docs"]

    # ---- parity spot-check of the timed outputs (rank 0 sample vs the CPU oracle)
    parity = None
    if rank == 0:
        import oracle
        n = args.docs
        torch.cuda.synchronize()
        off = _d2h(r.off, n * 8).view(np.uint64)
        ln = _d2h(r.len, n * 8).view(np.uint64)
        st = _d2h(r.status, n * 4).view(np.int32)
        hdata = _d2h(r.data, int(r.data_bytes)).tobytes()
        ups = synth.split(arena, upd_off)
        checked = 0
        for dd in range(0, n, max(1, n // 400)):
            exp = oracle.merge_updates(ups[doc_upd[dd]:doc_upd[dd + 1]])
            got = (int(st[dd]), hdata[int(off[dd]):int(off[dd]) + int(ln[dd])])
            assert exp == got, f"parity failure on document {dd}"
            checked += 1
        assert (st == 0).all()
        parity = f"bit-exact vs oracle on {checked} sampled docs; all {n} statuses OK"

    if rank == 0:
        value = all_bytes * args.steps / dt / 1e6
        achieved = algo_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None
        line = {
            "metric": "merged update MB/s (bit-exact vs yjs mergeUpdates)",
            "value": round(value, 3),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded V1 updates, tools/synth.c; SURVEY.md §8d C2)",
            "config": {"workload": f"C2: {args.docs} docs x {args.updates} single-char Y.Text insert updates per GPU, "
                                   "1-4 uint32 clients, batched Y.mergeUpdates, inputs resident in HBM",
                       "docs_per_gpu": args.docs, "updates_per_gpu": n_upd, "bytes_in_per_gpu": len(arena),
                       "bytes_out_per_gpu": out_bytes, "parallelism": f"doc-sharded x{world}"},
            "docs_per_s": round(all_docs * args.steps / dt, 1),
            "roofline": {"bound": "hbm", "kernel": "k_merge_lean (+ k_merge_wave / k_merge_fast / k_merge_big / k_merge_seq for deferred docs)",
                         "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 5) if achieved else None,
                         "kernel_ms": round(kernel_ms, 4), "traffic": _pmc_traffic()},
            "parity": parity,
            "seq_kernel_docs": node["docs_seq"],
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(arena, upd_off, doc_upd, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


def _d2h(src, n):
    """Copies n bytes of engine-owned device memory to a host numpy array."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.empty(max(n, 1), np.uint8)
    if n:
        assert hip.hipMemcpy(out.ctypes.data, src, n, 2) == 0  # hipMemcpyDeviceToHost
    return out[:n]


def _pmc_traffic():
    """HBM bytes per k_merge_wave launch (FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 --pmc passes of this
    same command; tools/prof_summary.py) from the committed profile, if any."""
    p = os.path.join(ROOT, "profiles", PMC_PROFILE)
    if os.path.exists(p):
        try:
            return json.load(open(p)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


if __name__ == "__main__":
    main()
