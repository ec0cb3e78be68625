"""Benchmark: batched Y.mergeUpdates / diffUpdate / encodeStateVectorFromUpdate on MI355X
(BASELINE.json metric "merged update MB/s + docs/sec (bit-exact vs yjs) at 1/2/4/8 MI355X").

    python bench.py [--gpus N] [--steps K] [--warmup W] [...]

One JSON line (rank 0).  Its headline (`value`, `roofline`, `cpu_baseline`) is config C2
(BASELINE.json configs[1]): 10 000 documents x 200 single-character Y.Text insert
updates per GPU, one step = one batched mergeUpdates over all of them with the inputs resident in
HBM (ygm_merge_v1_device_async: counter reset + the lean kernel; every C2 document is finished by
the lean kernel -- asserted -- so no step needs the host-driven tiers).  Beside it, as extra keys:

  c2_100k  the same merge at 100 000 documents per GPU (0.47 GB in: past the 256 MiB Infinity Cache,
           so the HBM fraction is not L3-served)
  c2_1m    the same merge over 1 000 000 documents in all (4.7 GB in, sharded over the ranks): the north_star size
  c4       config C4 (configs[3]): 1 000 000 merged Y.Text states (1-16 clients, log-uniform 1-8 KB,
           3.2 GB) sharded over the ranks, encodeStateVectorFromUpdate and diffUpdate against per-document
           state vectors (the mass-reconnect Step1 -> Step2 path, MessageReceiver.ts:137-155)
  c2_mixed C2 past the lean kernel's envelope: 1-8 clients, 1-16 character inserts, 20 % deletions (tier cascade)
  c3       config C3 at full size (configs[2]): 100 000 [snapshot, ...log] documents of 10 MB * rank^-0.8 (0.77 GB)
           merged in one batch through the tier cascade, beside the C port and yjs (rank 0 at N = 1)
  c5       config C5 at BASELINE size (configs[4]): 1 000 Y.XmlFragment [snapshot, ...log] documents of 10 000 client
           blocks each (0.29 GB), formats / embeds / attributes, merged in one batch, beside the C port and yjs
  c5_store the default product store at C5 size: 1 000 Tiptap-style [state, ...log] documents of 10 000 client blocks
           from a simulated session yjs integrates completely (tools/synth_live.c), merged, then normalized
           (encodeStateAsUpdate(applyUpdate(new Doc, merged)): what GpuMerge stores by default), each leg timed
  v2       SURVEY.md §8f-4: the C2 merge with the updates in format V2 (Y.mergeUpdatesV2), and the V1 <-> V2
           conversions of its 2 M updates
  cpu_baseline  the reference yjs path on the GPU box's host cores (yjs 13.5.16 from the image's
           JupyterLab bundle on Node worker_threads, kind "reference") with the C restatement
           (oracle/yjs_oracle.c on pthreads, kind "port") nested beside it; c4 carries its own

N > 1: one process per GPU.  Run directly as `python bench.py --gpus N` the script starts N rank
processes through torch.distributed.run before anything touches a GPU (and exits with their code);
under torchrun it reads RANK / LOCAL_RANK / WORLD_SIZE.  Documents are named ("c2-<i>", "c4-<i>") and
each rank takes those with fnv1a64(name) mod N == rank (hocuspocus_amd.shard): C2 is weak-scaled
(10 000 x N documents in all), C4 strong-scaled (1 000 000 in all).  No update data crosses GPUs: the
collectives are the barrier, the max-reduction of the timed spans and the node stats gather.

Algorithmic bytes: merge sum(|inputs|) + |output|; diff |u| + |sv| + |out|; state vector
|u| + |out|.  `roofline.achieved` = one launch's algorithmic bytes / its HIP-event time on the stream
it ran on; peak 8 TB/s (MI355X_MICROARCH.md).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
PMC_PROFILE = "r06_final/pmc.json"          # committed rocprofv3 PMC summary (FETCH_SIZE x2 + WRITE_SIZE per launch)
PMC_C4 = "r06_final/pmc.json"              # ... of the SV / diff walker at C4
PMC_BLOCKS = "r06_final/pmc_blocks.json"   # ... of whole blocks (--big, --block: every kernel of a step summed, tools/pmc_blocks.py)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=10000, help="C2 documents per GPU")
    ap.add_argument("--updates", type=int, default=200)
    ap.add_argument("--c2big-docs", type=int, default=100000, help="C2 documents per GPU of the c2_100k block (0: skip)")
    ap.add_argument("--c2m-docs", type=int, default=1000000, help="C2 documents in all of the c2_1m block (0: skip)")
    ap.add_argument("--c4-docs", type=int, default=1000000, help="C4 documents in all (0: skip)")
    ap.add_argument("--c4-steps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="budget of each CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads / workers (0: the cores granted: affinity mask, cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-yjs", action="store_true", help="skip the Node / yjs leg of the CPU baseline")
    ap.add_argument("--no-v2", dest="v2", action="store_false", help="skip the update-V2 (f-4) block")
    ap.add_argument("--no-c3", dest="c3", action="store_false", help="skip the full-size C3 block")
    ap.add_argument("--c5-docs", type=int, default=1000, help="documents of the C5 block (BASELINE size 1000; 0: skip)")
    ap.add_argument("--no-mixed", dest="mixed", action="store_false", help="skip the c2_mixed block")
    ap.add_argument("--f1-docs", type=int, default=10000, help="documents of the f1 (doc-normalized snapshot) block (0: skip)")
    ap.add_argument("--no-host-api", dest="host_api", action="store_false",
                    help="skip the host_api block (host arrays through the pinned / two-stream host API)")
    ap.add_argument("--big", choices=["c3", "c5", "c3full"], default=None,
                    help="instead of the standard line: one C3 / C5 large-document batch on the GPU next to the CPU oracle")
    ap.add_argument("--big-docs", type=int, default=None)
    ap.add_argument("--store-docs", type=int, default=1000, help="documents of the c5_store block (BASELINE C5 size 1000; 0: skip)")
    ap.add_argument("--block", choices=["f1", "mixed", "v2", "store"], default=None,
                    help="run one side block alone and print its JSON (counter passes: tools/pmc_blocks.py)")
    ap.add_argument("--dry-run", action="store_true", help="no GPU: gloo + the CPU oracle stand in (tests of the rank path)")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(args):
    """`python bench.py --gpus N` outside torchrun: N rank processes, started before any GPU call."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_cores(args):
    """CPU-baseline threads / Node workers = the cores the host grants this process (BASELINE north_star: "Node
    worker_threads = core count, stated"): the affinity mask, bounded by the cgroup CPU quota when one is set --
    on the GPU box the mask lists 256 CPUs but cpu.max grants 16 CPUs of time, and 256 workers time-sliced on
    16 CPUs measure the throttling, not the reference (r03 run: yjs merge 15 MB/s on 256 workers vs 113 MB/s on
    16).  Both numbers are stated beside every baseline (host_cpus()); --cpu-threads overrides."""
    if args.cpu_threads:
        return args.cpu_threads
    h = host_cpus()
    n = h["affinity"]
    if h["cgroup_cpu_quota"]:
        n = min(n, max(1, int(h["cgroup_cpu_quota"] + 0.999)))
    return max(1, n)


def host_cpus():
    """What the host grants, stated beside every CPU baseline: the affinity mask, os.cpu_count() and the
    cgroup CPU quota (cpu.max, in CPUs; null when unlimited or absent)."""
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = None if q <= 0 else round(q / per, 2)
        except Exception:
            pass
    return {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota}


# ----------------------------------------------------------------------------- backends
class GpuBackend:
    """Device-resident batches on one MI355X through the C ABI (include/ygm.h)."""

    def __init__(self, local):
        import torch
        from hocuspocus_amd import Engine
        self.torch = torch
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.eng = Engine(local)
        self.stream = torch.cuda.current_stream(self.dev)

    def put(self, a, pad=0):
        a = np.ascontiguousarray(a)
        if pad:
            a = np.concatenate([a.view(np.uint8).reshape(-1), np.zeros(pad, np.uint8)])
        return self.torch.from_numpy(a).to(self.dev)

    def merge_async(self, c):
        if "doff" in c:
            self.eng.merge_device_lens_async(c["da"], c["bytes"], c["doff"], c["dlen"], c["dd"], c["n_upd"], c["n"],
                                             self.stream.cuda_stream)
        else:
            self.eng.merge_device_async(c["da"], c["bytes"], c["do"], c["dd"], c["n_upd"], c["n"], self.stream.cuda_stream)

    def merge_finish(self):
        return self.eng.merge_device_finish()

    def sv(self, c):
        return self.eng.sv_device(c["da"], c["bytes"], c["do"], c["n"], self.stream.cuda_stream)

    def diff(self, c):
        return self.eng.diff_device(c["da"], c["bytes"], c["do"], c["ds"], c["dso"], c["n"], self.stream.cuda_stream)

    def sync(self):
        self.torch.cuda.synchronize()

    def stats(self):
        return self.eng.stats()

    def fetch(self, r, n):
        """(status, off, len, data bytes) of a device result."""
        self.sync()
        return (_d2h(r.status, n * 4).view(np.int32), _d2h(r.off, n * 8).view(np.uint64), _d2h(r.len, n * 8).view(np.uint64),
                _d2h(r.data, int(r.data_bytes)).tobytes())

    def close(self):
        self.eng.close()


class DryBackend:
    """--dry-run: the CPU oracle stands in for the engine (no timing meaning; tests the rank path)."""

    class _S:
        def __init__(self):
            self.kernel_ms = self.lean_ms = 0.0
            self.lean_launches = self.docs_lean = self.docs_seq = self.docs_fast = 0

    class _R:
        def __init__(self, payload):
            self.payload_bytes = payload

    def __init__(self):
        import oracle
        self.o = oracle
        self.s = self._S()
        self.last = None

    def put(self, a, pad=0):
        return np.ascontiguousarray(a)

    def _t(self, f, launches, docs):
        t0 = time.perf_counter()
        r = f()
        ms = (time.perf_counter() - t0) * 1e3
        self.s.kernel_ms += ms
        self.s.lean_ms += ms
        self.s.lean_launches += launches
        self.s.docs_lean += docs
        return r

    def merge_async(self, c):
        st, algo = self._t(lambda: self.o.merge_batch(c["da"], c["do"], c["dd"], 1), 1, 0)
        self.last = self._R(algo - c["bytes"])
        self.last_n = c["n"]

    def merge_finish(self):   # (the engine counts a span's documents once, at its finish)
        self.s.docs_lean += self.last_n
        return self.last

    def sv(self, c):
        st, algo = self._t(lambda: self.o.doc_batch("sv", c["da"], c["do"], threads=1), 1, c["n"])
        return self._R(algo - c["bytes"])

    def diff(self, c):
        st, algo = self._t(lambda: self.o.doc_batch("diff", c["da"], c["do"], c["ds"], c["dso"], threads=1), 1, c["n"])
        return self._R(algo - c["bytes"] - c["sv_bytes"])

    def sync(self):
        pass

    def stats(self):
        import copy
        return copy.copy(self.s)

    def close(self):
        pass


def _d2h(src, n):
    """Copies n bytes of engine-owned device memory to a host numpy array."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.empty(max(n, 1), np.uint8)
    if n:
        assert hip.hipMemcpy(out.ctypes.data, src, n, 2) == 0  # hipMemcpyDeviceToHost
    return out[:n]


def _pmc(name, key):
    """HBM bytes per launch of a kernel (FETCH_SIZE x2 + WRITE_SIZE from separate rocprofv3 --pmc passes,
    MI355X_MICROARCH.md §HBM) from the committed profile summary, if any."""
    p = os.path.join(ROOT, "profiles", name)
    try:
        d = json.load(open(p))
        return d.get(key) if key else d.get("hbm_bytes_per_launch")
    except Exception:
        return None


# ----------------------------------------------------------------------------- workloads
def c2_corpus(be, prefix, per_gpu, updates, rank, world):
    from tools import synth
    idx = synth.partition(prefix, per_gpu * world, world, rank)
    arena, upd_off, doc_upd = synth.text_updates_docs(idx, updates)
    c = {"arena": arena, "upd_off": upd_off, "doc_upd": doc_upd, "n": len(idx), "n_upd": int(doc_upd[-1]), "bytes": len(arena)}
    c["da"] = be.put(arena, 64)
    c["do"] = be.put(upd_off.view(np.int64))
    c["dd"] = be.put(doc_upd.view(np.int32))
    lens = np.diff(upd_off.astype(np.int64))
    if isinstance(be, GpuBackend) and lens.max(initial=0) < 65536:
        # the compact input form (include/ygm.h ygm_merge_v1_device_lens): u64 per document + u16 per update
        c["doff"] = be.put(upd_off[doc_upd].view(np.int64))
        c["dlen"] = be.put(lens.astype(np.uint16).view(np.int16))
    return c


def _host_stats(e):
    s = e.stats()
    return {"kernel_ms": s.kernel_ms, "h2d_ms": s.h2d_ms, "d2h_ms": s.d2h_ms}


def host_api_merge(be, cb, args, reps=3):
    """The production path: host arrays through ygm_merge_v1 (pinned staging, two stage streams, device-side packing,
    D2H of the packed outputs) -- what the N-API addon and GpuMerge call.  End-to-end rate = algorithmic bytes / wall."""
    from hocuspocus_amd import Engine
    import oracle
    e = Engine(be.dev.index)
    arena, upd_off, doc_upd = cb["arena"], cb["upd_off"], cb["doc_upd"]
    upd_doc = np.repeat(np.arange(cb["n"], dtype=np.uint32), np.diff(doc_upd.astype(np.int64)))
    e.merge_packed_raw(arena, upd_off, upd_doc, cb["n"])   # warm-up: stage contexts, pinned buffers
    s0 = _host_stats(e)
    t0 = time.perf_counter()
    for _ in range(reps):
        st, off, ln, data = e.merge_packed_raw(arena, upd_off, upd_doc, cb["n"])
    wall = (time.perf_counter() - t0) / reps
    s1 = _host_stats(e)
    out_b = int(ln.sum())
    ok = 0
    for d in range(0, cb["n"], max(1, cb["n"] // 200)):
        ups = [arena[upd_off[u]:upd_off[u + 1]].tobytes() for u in range(doc_upd[d], doc_upd[d + 1])]
        got = (int(st[d]), bytes(data[int(off[d]):int(off[d]) + int(ln[d])]) if st[d] == 0 else None)
        assert oracle.merge_updates(ups) == got, f"host API parity failure on document {d}"
        ok += 1
    d = {k: (s1[k] - s0[k]) / reps for k in s0}
    h2d_b = len(arena) + upd_off.nbytes + 4 * (cb["n"] + 1)
    d2h_b = out_b + 20 * cb["n"]
    e.close()
    return {"op": "merge (ygm_merge_v1, host arrays)", "docs": cb["n"], "value": round((len(arena) + out_b) / wall / 1e6, 1),
            "unit": "MB/s end-to-end (algorithmic bytes / wall, PCIe + host staging included)", "wall_ms": round(wall * 1e3, 3),
            "docs_per_s": round(cb["n"] / wall, 1), "h2d_ms": round(d["h2d_ms"], 3), "d2h_ms": round(d["d2h_ms"], 3),
            "device_span_ms": round(d["kernel_ms"], 3), "h2d_bytes": int(h2d_b), "d2h_bytes": int(d2h_b),
            "h2d_GBps": round(h2d_b / max(d["h2d_ms"], 1e-6) / 1e6, 2), "d2h_GBps": round(d2h_b / max(d["d2h_ms"], 1e-6) / 1e6, 2),
            "pipeline": "64 MB chunks of whole documents over two stage streams: pinned staging + H2D of chunk i+1 beside the "
                        "kernels of chunk i, device-side packing, D2H of packed outputs",
            "parity": f"bit-exact vs oracle on {ok} sampled docs"}


def c1_store_window(docs=1000, inserts=200):
    """C1: one store window of 1 000 edited Y.Text documents through GpuMerge (Node, N-API addon:
    ygm_merge_v1, then ygm_snapshot_v1 -- the default normalized store; and normalize: false, the merge alone)
    beside extension-database's encodeStateAsUpdate store (tools/c1_store_latency.js)."""
    import shutil
    import subprocess
    if not shutil.which("node"):
        return {"skipped": "node not found"}
    try:
        r = subprocess.run(["node", os.path.join(ROOT, "tools", "c1_store_latency.js"), str(docs), str(inserts)],
                           capture_output=True, text=True, timeout=240)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        return json.loads(lines[-1]) if r.returncode == 0 and lines else {"error": (r.stderr or r.stdout)[-400:]}
    except Exception as ex:   # the block is a report, not the headline: keep the line
        return {"error": repr(ex)[:400]}


def f1_block(be, args, steps=5):
    """snapshot(u) = encodeStateAsUpdate(applyUpdate(new Doc, u)) -- what extension-database stores --
    over the merged states of C2 logs with 20 % deletions (the GpuMerge normalize path: merge, then snapshot).
    Inputs resident in HBM; per step the count + scan + snapshot kernels (one workspace-size read between them)."""
    from hocuspocus_amd import Engine
    from tools import synth
    e = Engine(be.dev.index, compat135=True)
    arena, upd_off, doc_upd = synth.text_updates(args.f1_docs, args.updates, seed=61, del_pct=20)
    upd_doc = np.repeat(np.arange(args.f1_docs, dtype=np.uint32), np.diff(doc_upd.astype(np.int64)))
    st, off, ln, data = e.merge_packed_raw(arena, upd_off, upd_doc, args.f1_docs)
    assert (st == 0).all()
    buf = np.frombuffer(bytes(data), np.uint8)
    states = np.concatenate([buf[int(off[d]):int(off[d]) + int(ln[d])] for d in range(args.f1_docs)])
    doc_off = np.zeros(args.f1_docs + 1, np.uint64)
    doc_off[1:] = np.cumsum(ln.astype(np.uint64))
    da, do = be.put(states, 64), be.put(doc_off.view(np.int64))
    for _ in range(2):
        e.snapshot_device(da, len(states), do, args.f1_docs, be.stream.cuda_stream)
    s0 = e.stats()
    be.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = e.snapshot_device(da, len(states), do, args.f1_docs, be.stream.cuda_stream)
    be.sync()
    wall = (time.perf_counter() - t0) / steps
    s1 = e.stats()
    kms = (s1.kernel_ms - s0.kernel_ms) / steps
    algo = len(states) + int(r.payload_bytes)
    stat = _d2h(r.status, 4 * args.f1_docs).view(np.int32)
    blk = {"workload": f"f-1: {args.f1_docs} C2 logs ({args.updates} single-char updates, 20 % deletions, 1-4 clients) merged, then "
                       "snapshotted (YATA integrate + GC + merge + encode, yjs 13.5.16 semantics), inputs resident in HBM",
           "docs": args.f1_docs, "bytes_in": len(states), "bytes_out": int(r.payload_bytes), "ok_docs": int((stat == 0).sum()),
           "value": round(algo / kms / 1e3, 3), "unit": "MB/s", "docs_per_s": round(args.f1_docs / kms * 1e3, 1),
           "ms_per_step": round(kms, 4), "wall_ms_per_step": round(wall * 1e3, 4),
           "roofline": roof(algo, kms, "k_snap_text (flat text: one document per wave, workspace in LDS) + k_snap_count / scan / k_snap "
                                        "(one thread per document) for what it leaves", _pmc(PMC_BLOCKS, "f1")),
           "parity": "yjs vectors in tests/test_snapshot.py (440 fixed + live sessions + GPU-merged C2 logs) -- bit-exact"}
    if not args.no_cpu_baseline and not args.no_yjs:
        c = {"arena": states, "doc_off": doc_off}
        blk["cpu_baseline"] = cpu_yjs("snapshot", c, cpu_cores(args), min(args.f1_docs, 4000))
    e.close()
    return blk


def store_block(be, args, steps=2):
    """The default product store at BASELINE config C5's size: what GpuMerge stores for each document --
    Y.mergeUpdates([state, ...log]) on the GPU, then the doc-normalized snapshot encodeStateAsUpdate(applyUpdate(new
    Doc, merged)) for merged states up to normalizeMaxBytes (32 KiB, packages/extension-gpu-merge/src/index.js) and the
    bare merge above it (extension-database Database.ts:55-60, extension-s3 S3.ts:92-103) -- over 1 000 Tiptap-style
    XmlFragment documents of 10 000 client blocks each (tools/synth_live.c: a simulated session yjs integrates
    completely; the C5 merge corpus of tools/synth.c is not loadable by Y.applyUpdate).  Timed legs, inputs resident in
    HBM: the merge of the 1 000 batches; the snapshot of the documents under the limit (none at this size); and, as
    the cost the limit avoids, the forced snapshot of a sample (the snapshot kernel runs a document on one thread)."""
    from hocuspocus_amd import Engine
    import oracle
    from tools import synth
    n, limit = args.store_docs, 32768

    def note(msg):   # progress on stderr (a long block must not look hung)
        print(f"[c5_store] {msg}", file=sys.stderr, flush=True)
    arena, upd_off, doc_upd = synth.live_docs(n, 1_000_000, 64 * 1024, n_clients=10000, max_k=50, xml=True, seed=9)
    note(f"{n} documents, {len(arena) / 1e6:.1f} MB")
    e = Engine(be.dev.index)   # the 13.6 default (GpuMerge's): the large-document tier unions multi-client delete sets
    da, do, dd = be.put(arena, 64), be.put(upd_off.view(np.int64)), be.put(doc_upd.view(np.int32))
    n_upd = int(doc_upd[-1])
    mms, tiers = [], None
    for it in range(steps + 1):   # the first run grows the scratch
        s0 = e.stats()
        r = e.merge_device(da, len(arena), do, dd, n_upd, n, be.stream.cuda_stream)
        s1 = e.stats()
        if it:
            mms.append(s1.kernel_ms - s0.kernel_ms)
        tiers = {"big": s1.docs_big - s0.docs_big, "seq": s1.docs_seq - s0.docs_seq}
        note(f"merge run {it}: {s1.kernel_ms - s0.kernel_ms:.1f} ms, tiers {tiers}")
    st, off, ln, data = be.fetch(r, n)
    assert (st == 0).all()
    merged_bytes = int(ln.sum())
    ups = synth.split(arena, upd_off)
    checked = 0
    for d in sorted(set([0, 1, n - 1] + list(range(0, n, max(1, n // 20))))):   # merge parity on a sample
        assert oracle.merge_updates(ups[doc_upd[d]:doc_upd[d + 1]]) == (0, data[int(off[d]):int(off[d]) + int(ln[d])]), d
        checked += 1
    states = [np.frombuffer(data[int(off[d]):int(off[d]) + int(ln[d])], np.uint8) for d in range(n)]

    def snap(docs, reps):   # kernel ms (best of reps) and output bytes of ygm_snapshot_v1_device over `docs`
        if not docs:
            return 0.0, 0, 0
        cat = np.concatenate([states[d] for d in docs])
        doff = np.zeros(len(docs) + 1, np.uint64)
        doff[1:] = np.cumsum([len(states[d]) for d in docs])
        ds, dso = be.put(cat, 64), be.put(doff.view(np.int64))
        best, rs = None, None
        for _ in range(reps):
            s0 = e.stats()
            rs = e.snapshot_device(ds, len(cat), dso, len(docs), be.stream.cuda_stream)
            be.sync()
            ms = e.stats().kernel_ms - s0.kernel_ms
            best = ms if best is None or ms < best else best
        ok = int((_d2h(rs.status, 4 * len(docs)).view(np.int32) == 0).sum())
        return best, int(rs.payload_bytes), ok
    under = [d for d in range(n) if len(states[d]) <= limit]
    sms, sout, sok = snap(under, 2)
    over_bytes = sum(len(states[d]) for d in range(n) if len(states[d]) > limit)
    note(f"forced snapshot of all {n} documents")
    sample = list(range(n))
    fms, fout, fok = snap(sample, 1)
    note(f"forced snapshot: {fms:.1f} ms")
    stored = sout + over_bytes
    mm = sorted(mms)[len(mms) // 2]
    total_ms = mm + sms
    blk = {"workload": f"default product store at C5 size: {n} Y.XmlFragment [state, ...log] documents, 10 000 client blocks each "
                       f"(tools/synth_live.c), Y.mergeUpdates then the snapshot for merged states <= {limit} bytes (GpuMerge "
                       f"normalizeMaxBytes), inputs resident in HBM",
           "docs": n, "bytes_in": len(arena), "merged_bytes": merged_bytes, "stored_bytes": stored,
           "largest_doc": int(max(len(x) for x in states)), "merge_tiers": tiers,
           "docs_normalized": len(under), "docs_over_limit": n - len(under),
           "merge_ms": round(mm, 3), "snapshot_ms": round(sms, 3), "ms_per_step": round(total_ms, 3),
           "value": round((len(arena) + stored) / total_ms / 1e3, 3), "unit": "MB/s", "docs_per_s": round(n / total_ms * 1e3, 1),
           "roofline": roof(len(arena) + merged_bytes, mm, "merge cascade (large-document tier)", _pmc(PMC_BLOCKS, "c5_store")),
           "forced_snapshot_all": {"docs": len(sample), "bytes_in": int(sum(len(states[d]) for d in sample)), "bytes_out": fout,
                                   "ok_docs": fok, "ms": round(fms, 1), "MBps": round(sum(len(states[d]) for d in sample) / fms / 1e3, 1),
                                   "us_per_byte_largest": round(fms * 1e3 / max(len(states[d]) for d in sample), 2),
                                   "note": "normalize: every document snapshotted, encodeStateAsUpdate(applyUpdate(new Doc, merged)) "
                                           "on the GPU: one thread per document, so the batch takes its largest document's time"},
           "parity": f"merge: bit-exact vs oracle on {checked} documents; snapshot: tests/test_snapshot.py::"
                     "test_gpu_snapshot_at_baseline_sizes (yjs 13.5.16 on the box)"}
    if not args.no_cpu_baseline and not args.no_yjs:
        k = min(n, 100)
        blk["cpu_baseline"] = {"merge": cpu_yjs("merge", {"arena": arena, "upd_off": upd_off, "doc_upd": doc_upd}, cpu_cores(args), k)}
        ks = min(n, 64)
        cat = np.concatenate(states[:ks])
        doff = np.zeros(ks + 1, np.uint64)
        doff[1:] = np.cumsum([len(x) for x in states[:ks]])
        blk["cpu_baseline"]["snapshot"] = cpu_yjs("snapshot", {"arena": cat, "doc_off": doff}, cpu_cores(args), ks)
    e.close()
    return blk


def mixed_block(be, args, steps=5):
    """C2 past the lean kernel's envelope (realistic debounce logs): 10 000 documents x 200 updates
    of 1-8 clients (uint32 ids), inserts of 1-16 characters as one Item (pastes, words typed in one transaction:
    updates of up to ~42 bytes) and 20 % deletions -- one batched merge per step through the whole tier cascade
    (documents the lean kernel cannot prove go on to the wave / workgroup tiers), inputs resident in HBM."""
    from hocuspocus_amd import Engine
    import oracle
    from tools import synth
    n = args.docs
    arena, upd_off, doc_upd = synth.text_updates(n, args.updates, 1, 8, del_pct=20, seed=71, max_run=16)
    e = Engine(be.dev.index)
    da, do, dd = be.put(arena, 64), be.put(upd_off.view(np.int64)), be.put(doc_upd.view(np.int32))
    n_upd = int(doc_upd[-1])
    r = e.merge_device(da, len(arena), do, dd, n_upd, n, be.stream.cuda_stream)
    be.sync()
    s0 = e.stats()
    for _ in range(steps):
        r = e.merge_device(da, len(arena), do, dd, n_upd, n, be.stream.cuda_stream)
    be.sync()
    s1 = e.stats()
    kms = (s1.kernel_ms - s0.kernel_ms) / steps
    algo = len(arena) + int(r.payload_bytes)
    st, off, ln, data = be.fetch(r, n)
    ups = synth.split(arena, upd_off)
    checked = 0
    for d in range(0, n, max(1, n // 200)):
        exp = oracle.merge_updates(ups[doc_upd[d]:doc_upd[d + 1]])
        assert exp == (int(st[d]), data[int(off[d]):int(off[d]) + int(ln[d])] if st[d] == 0 else None), f"parity failure on document {d}"
        checked += 1
    e.close()
    return {"workload": f"C2 mixed: {n} docs x {args.updates} updates, 1-8 uint32 clients, 1-16 character inserts, 20 % deletions "
                        "(updates up to ~42 bytes), batched Y.mergeUpdates through the tier cascade, inputs resident in HBM",
            "docs": n, "bytes_in": len(arena), "bytes_out": int(r.payload_bytes), "value": round(algo / kms / 1e3, 3), "unit": "MB/s",
            "docs_per_s": round(n / kms * 1e3, 1), "ms_per_step": round(kms, 4),
            "docs_lean": int((s1.docs_lean - s0.docs_lean) / steps), "docs_lean_wide": int((s1.docs_lean_wide - s0.docs_lean_wide) / steps),
            "docs_general_tiers": int((s1.docs_fast - s0.docs_fast) / steps),
            "docs_big": int((s1.docs_big - s0.docs_big) / steps), "docs_seq": int((s1.docs_seq - s0.docs_seq) / steps),
            "roofline": roof(algo, kms, "k_merge_lean<1> (wide route: the batch's average document outgrows the narrow kernel's "
                                        "staging) + the general tiers for its deferrals", _pmc(PMC_BLOCKS, "c2_mixed")),
            "parity": f"bit-exact vs oracle on {checked} sampled docs"}


def v2_block(be, args, steps=5):
    """the C2 headline workload in update format V2 (the updates converted from the C2 V1 corpus by
    ygm_convert_v1_to_v2): Y.mergeUpdatesV2 per document, inputs resident in HBM.  Per step: the V2 -> V1 transcoding
    kernels, the V1 merge cascade, the V1 -> V2 kernels (two size reads between them); plus the conversions alone."""
    from hocuspocus_amd import Engine
    import oracle
    from tools import synth
    e = Engine(be.dev.index)
    idx = synth.partition("c2-", args.docs, 1, 0)
    a1, o1, d1 = synth.text_updates_docs(idx, args.updates)
    n, n_upd = len(idx), int(d1[-1])
    st, off, ln, data = e._raw(e._conv_packed("ygm_convert_v1_to_v2", a1, o1))
    assert (st == 0).all()
    o2 = np.zeros(n_upd + 1, np.uint64)
    o2[1:] = np.cumsum(ln.astype(np.uint64))
    assert (np.asarray(off, np.uint64) == o2[:-1]).all()   # the host API packs outputs in order, without gaps
    a2 = np.frombuffer(bytes(data), np.uint8)[:int(o2[-1])].copy()
    da, do, dd = be.put(a2, 64), be.put(o2.view(np.int64)), be.put(d1.view(np.int32))
    r = e.merge_v2_device(da, len(a2), do, dd, n_upd, n, be.stream.cuda_stream)
    be.sync()
    s0 = e.stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = e.merge_v2_device(da, len(a2), do, dd, n_upd, n, be.stream.cuda_stream)
    be.sync()
    wall = (time.perf_counter() - t0) / steps
    s1 = e.stats()
    kms = (s1.kernel_ms - s0.kernel_ms) / steps
    algo = len(a2) + int(r.payload_bytes)
    st2, off2, ln2, out2 = be.fetch(r, n)
    ups2 = synth.split(a2, o2)
    checked = 0
    for d in range(0, n, max(1, n // 100)):
        exp = oracle.merge_updates_v2(ups2[d1[d]:d1[d + 1]])
        assert exp == (int(st2[d]), out2[int(off2[d]):int(off2[d]) + int(ln2[d])]), f"V2 parity failure on document {d}"
        checked += 1
    conv = {}
    a1d, o1d = be.put(a1, 64), be.put(o1.view(np.int64))
    for op, (da_, do_, nb) in (() if args.block else (("v1_to_v2", (a1d, o1d, len(a1))), ("v2_to_v1", (da, do, len(a2))))):
        e.doc_v2_device(op, da_, nb, do_, n_upd, stream=be.stream.cuda_stream)
        be.sync()
        c0 = e.stats()
        rr = e.doc_v2_device(op, da_, nb, do_, n_upd, stream=be.stream.cuda_stream)
        be.sync()
        cms = e.stats().kernel_ms - c0.kernel_ms
        conv[op] = {"updates": n_upd, "ms": round(cms, 4), "value": round((nb + int(rr.payload_bytes)) / cms / 1e3, 3), "unit": "MB/s"}
    blk = {"workload": f"C2 in update format V2: {n} docs x {args.updates} updates (V2, {len(a2)} bytes; the V1 corpus is "
                       f"{len(a1)} bytes), batched Y.mergeUpdatesV2, inputs resident in HBM",
           "docs": n, "updates": n_upd, "bytes_in": len(a2), "bytes_out": int(r.payload_bytes),
           "value": round(algo / kms / 1e3, 3), "unit": "MB/s", "docs_per_s": round(n / kms * 1e3, 1), "ms_per_step": round(kms, 4),
           "wall_ms_per_step": round(wall * 1e3, 4),
           "roofline": roof(algo, kms, "k_v21f (lane per update, column decoders in registers) + V1 merge cascade + k_v12_fast "
                                        "(a V2 column per lane)", _pmc(PMC_BLOCKS, "v2")),
           "convert": conv, "parity": f"bit-exact vs oracle (yjs_oracle_v2.c) on {checked} sampled docs; tests/test_v2.py: 4887 yjs vectors"}
    if not args.no_cpu_baseline and not args.no_yjs:
        blk["cpu_baseline"] = cpu_yjs("merge_v2", {"arena": a2, "upd_off": o2, "doc_upd": d1}, cpu_cores(args), min(n, 4000))
    e.close()
    return blk


def host_api_doc(be, c, op, n, reps=3):
    from hocuspocus_amd import Engine
    import oracle
    e = Engine(be.dev.index)
    arena = c["arena"][:int(c["doc_off"][n])]
    doc_off = np.ascontiguousarray(c["doc_off"][:n + 1])
    sva = c["sva"][:int(c["sv_off"][n])]
    sv_off = np.ascontiguousarray(c["sv_off"][:n + 1])
    e.doc_packed_raw(op, arena, doc_off, sva, sv_off)
    s0 = _host_stats(e)
    t0 = time.perf_counter()
    for _ in range(reps):
        st, off, ln, data = e.doc_packed_raw(op, arena, doc_off, sva, sv_off)
    wall = (time.perf_counter() - t0) / reps
    s1 = _host_stats(e)
    out_b = int(ln.sum())
    ok = 0
    for d in range(0, n, max(1, n // 200)):
        u = arena[doc_off[d]:doc_off[d + 1]].tobytes()
        exp = oracle.diff_update(u, sva[sv_off[d]:sv_off[d + 1]].tobytes()) if op == "diff" else oracle.encode_state_vector_from_update(u)
        assert exp == (int(st[d]), bytes(data[int(off[d]):int(off[d]) + int(ln[d])]) if st[d] == 0 else None), f"host API parity failure {d}"
        ok += 1
    d = {k: (s1[k] - s0[k]) / reps for k in s0}
    algo = len(arena) + len(sva) + out_b
    e.close()
    return {"op": f"{op} (host arrays)", "docs": n, "value": round(algo / wall / 1e6, 1), "unit": "MB/s end-to-end",
            "wall_ms": round(wall * 1e3, 3), "docs_per_s": round(n / wall, 1), "h2d_ms": round(d["h2d_ms"], 3),
            "d2h_ms": round(d["d2h_ms"], 3), "device_span_ms": round(d["kernel_ms"], 3), "parity": f"bit-exact vs oracle on {ok} sampled docs"}


def time_merge(be, c, steps, warmup, dist):
    """Back-to-back async merges of the whole shard; returns (wall s, kernel ms per launch, payload, stats delta)."""
    w0 = be.stats()
    for _ in range(max(warmup, 1)):
        be.merge_async(c)
        be.merge_finish()
    be.sync()
    s0 = be.stats()
    assert s0.docs_lean - w0.docs_lean == c["n"] * max(warmup, 1), "not every document takes the lean kernel"
    if dist:
        dist.barrier()
    be.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        be.merge_async(c)
    be.sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    r = be.merge_finish()
    s1 = be.stats()
    assert s1.docs_lean - s0.docs_lean == c["n"], "a timed step deferred documents to the host-driven tiers"
    kms = (s1.lean_ms - s0.lean_ms) / max(s1.lean_launches - s0.lean_launches, 1)
    return dt, kms, int(r.payload_bytes), r


def time_doc(be, c, op, steps, dist):
    """SV or diff over the whole shard, `steps` times after one warmup; kernel time from the engine's HIP events."""
    f = be.sv if op == "sv" else be.diff
    f(c)
    be.sync()
    if dist:
        dist.barrier()
    s0 = be.stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = f(c)
    be.sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    s1 = be.stats()
    return dt, (s1.kernel_ms - s0.kernel_ms) / steps, r, s1.docs_lean - s0.docs_lean, s1.docs_fast - s0.docs_fast


def allmax(x, dist, dev):
    if not dist:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allsum(xs, dist, dev):
    if not dist:
        return list(xs)
    import torch
    t = torch.tensor([float(x) for x in xs], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def roof(algo_bytes, kernel_ms, kernel, traffic):
    a = algo_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None
    return {"bound": "hbm", "kernel": kernel, "achieved": round(a, 2) if a else None, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(a / HBM_PEAK_GBPS, 5) if a else None, "kernel_ms": round(kernel_ms, 4), "traffic": traffic}


# ----------------------------------------------------------------------------- CPU baselines
def cpu_port_merge(c, cores, budget_s):
    """oracle/yjs_oracle.c yo_merge_batch (literal C restatement of yjs mergeUpdates incl. V8 TimSort) on a bounded sample."""
    import oracle
    n = c["n"]

    def run(k, threads):
        t0 = time.perf_counter()
        st, algo = oracle.merge_batch(c["arena"], c["upd_off"], c["doc_upd"][:k + 1], threads)
        return time.perf_counter() - t0, algo, st

    n0 = min(n, 200)
    dt0, _, _ = run(n0, 1)
    sample = int(min(n, max(n0, budget_s * cores / max(dt0 / n0, 1e-9))))
    dt = algo = reps = 0
    while reps == 0 or dt * cores < budget_s:
        t, a, st = run(sample, cores)
        assert (st == 0).all()
        dt += t; algo += a; reps += 1
    return {"value": round(algo / dt / 1e6, 3), "unit": "MB/s", "cores": cores, "host": host_cpus(), "kind": "port", "docs_per_s": round(sample * reps / dt, 1),
            "sample": f"{reps} pass(es) over {sample} of the {n} C2 documents through oracle/yjs_oracle.c yo_merge_batch "
                      f"(C restatement of yjs mergeUpdates), {cores} pthreads, {dt:.2f} s wall"}


def cpu_port_doc(c, op, cores, k):
    """oracle/yjs_oracle.c yo_doc_batch (C restatement of encodeStateVectorFromUpdate / diffUpdate) over the first k documents."""
    import oracle
    t0 = time.perf_counter()
    if op == "diff":
        st, algo = oracle.doc_batch("diff", c["arena"], c["doc_off"][:k + 1], c["sva"], c["sv_off"][:k + 1], threads=cores)
    else:
        st, algo = oracle.doc_batch("sv", c["arena"], c["doc_off"][:k + 1], threads=cores)
    dt = time.perf_counter() - t0
    return {"value": round(algo / dt / 1e6, 3), "unit": "MB/s", "cores": cores, "host": host_cpus(), "kind": "port", "docs_per_s": round(k / dt, 1),
            "sample": f"the first {k} C4 documents through oracle/yjs_oracle.c yo_doc_batch, {cores} pthreads, {dt:.2f} s wall"}


def cpu_yjs(kind, c, cores, k):
    """yjs 13.5.16 (the image's JupyterLab bundle) on Node worker_threads = cores, over the first k documents."""
    import shutil
    import tempfile
    if shutil.which("node") is None:
        return None
    d = tempfile.mkdtemp(prefix="ygm_yjs_")
    try:
        if kind.startswith("merge"):
            u_end = int(c["doc_upd"][k])
            c["arena"][:int(c["upd_off"][u_end])].tofile(os.path.join(d, "arena.bin"))
            c["upd_off"][:u_end + 1].astype(np.uint64).tofile(os.path.join(d, "off.bin"))
            c["doc_upd"][:k + 1].astype(np.uint32).tofile(os.path.join(d, "docs.bin"))
        else:
            c["arena"][:int(c["doc_off"][k])].tofile(os.path.join(d, "arena.bin"))
            c["doc_off"][:k + 1].astype(np.uint64).tofile(os.path.join(d, "off.bin"))
            if kind == "diff":
                c["sva"][:int(c["sv_off"][k])].tofile(os.path.join(d, "sv.bin"))
                c["sv_off"][:k + 1].astype(np.uint64).tofile(os.path.join(d, "svoff.bin"))
        r = subprocess.run(["node", os.path.join(ROOT, "tools", "yjs_cpu_baseline.js"), d, kind, str(cores)], capture_output=True,
                           text=True, timeout=600)
        if r.returncode != 0:
            return {"error": r.stderr[-300:]}
        j = json.loads(r.stdout.strip().splitlines()[-1])
        ver = subprocess.run(["node", "--version"], capture_output=True, text=True).stdout.strip()
        return {"value": round(j["algo_bytes"] / j["seconds"] / 1e6, 3), "unit": "MB/s", "cores": cores, "host": host_cpus(), "kind": "reference",
                "docs_per_s": round(k / j["seconds"], 1),
                "sample": f"yjs 13.5.16 (JupyterLab bundle in the image; the reference pins 13.6.26) Y."
                          f"{ {'merge': 'mergeUpdates', 'merge_v2': 'mergeUpdatesV2', 'sv': 'encodeStateVectorFromUpdate', 'diff': 'diffUpdate', 'snapshot': 'encodeStateAsUpdate(applyUpdate(new Doc, u))'}[kind]} over the first "
                          f"{k} documents on Node {ver} worker_threads x {cores} (one per granted core), op loops only "
                          f"(common start barrier to the last worker's end) {j['seconds']:.2f} s"}
    finally:
        shutil.rmtree(d, ignore_errors=True)


# ----------------------------------------------------------------------------- the rank
def run_rank(args, rank, world, dist, be, dev=None):
    from hocuspocus_amd.shard import gather_stats
    # ---- headline: C2 merge, 10 000 documents per GPU
    c = c2_corpus(be, "c2-", args.docs, args.updates, rank, world)
    dt, kms, out_bytes, r = time_merge(be, c, args.steps, args.warmup, dist)
    algo = c["bytes"] + out_bytes
    dt = allmax(dt, dist, dev)
    node = gather_stats({"docs": c["n"], "updates": c["n_upd"], "bytes_in": c["bytes"], "bytes_out": out_bytes, "kernel_ms": kms}, dist, dev)
    parity = None
    if rank == 0 and not args.dry_run:
        import oracle
        from tools import synth
        st, off, ln, data = be.fetch(r, c["n"])
        ups = synth.split(c["arena"], c["upd_off"])
        checked = 0
        for d in range(0, c["n"], max(1, c["n"] // 400)):
            exp = oracle.merge_updates(ups[c["doc_upd"][d]:c["doc_upd"][d + 1]])
            assert exp == (int(st[d]), data[int(off[d]):int(off[d]) + int(ln[d])]), f"parity failure on C2 document {d}"
            checked += 1
        assert (st == 0).all()
        parity = f"bit-exact vs oracle on {checked} sampled docs; all {c['n']} statuses OK"
    line = None
    if rank == 0:
        value = (node["bytes_in"] + node["bytes_out"]) * args.steps / dt / 1e6
        line = {
            "metric": "merged update MB/s (bit-exact vs yjs mergeUpdates)",
            "value": round(value, 3), "unit": "MB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded V1 updates from per-document PRNG streams, tools/synth.c; SURVEY.md §8d C2)",
            "config": {"workload": f"C2: {args.docs} docs x {args.updates} single-char Y.Text insert updates per GPU (documents "
                                   f"'c2-<i>', i < {args.docs * world}, sharded by fnv1a64(name) mod {world}), 1-4 uint32 clients, "
                                   "batched Y.mergeUpdates, inputs resident in HBM",
                       "docs_per_gpu": args.docs, "docs_total": int(node["docs"]), "updates_total": int(node["updates"]),
                       "bytes_in_total": int(node["bytes_in"]), "bytes_out_total": int(node["bytes_out"]),
                       "parallelism": f"doc-sharded x{world}"},
            "docs_per_s": round(node["docs"] * args.steps / dt, 1),
            "roofline": roof(algo, kms, "k_merge_lean (rank 0; every C2 document is finished by it)", _pmc(PMC_PROFILE, None)),
            "parity": parity,
        }
    del c
    # ---- C2 at 100 000 documents per GPU (past the Infinity Cache)
    if args.c2big_docs:
        cb = c2_corpus(be, "c2b-", args.c2big_docs, args.updates, rank, world)
        dtb, kmsb, outb, _ = time_merge(be, cb, max(args.steps // 2, 1), 1, dist)
        dtb = allmax(dtb, dist, dev)
        tot = allsum([cb["n"], cb["bytes"] + outb], dist, dev)
        if rank == 0:
            sb = max(args.steps // 2, 1)
            line["c2_100k"] = {"docs_per_gpu": args.c2big_docs, "docs_total": int(tot[0]), "steps": sb,
                               "value": round(tot[1] * sb / dtb / 1e6, 3), "unit": "MB/s", "docs_per_s": round(tot[0] * sb / dtb, 1),
                               "ms_per_step": round(dtb / sb * 1e3, 4),
                               "roofline": roof(cb["bytes"] + outb, kmsb, "k_merge_lean (rank 0)", _pmc(PMC_C4, "k_merge_lean@100k"))}
        if rank == 0 and not args.dry_run and args.host_api:
            line["host_api"] = host_api_merge(be, cb, args)
            line["host_api"]["c1_store_window"] = c1_store_window()
        del cb
    # ---- C2 shape at 1M documents in all (north_star: "mergeUpdates ... over 1M synthetic documents"), 4.7 GB
    if args.c2m_docs:
        from tools import synth
        idx = synth.partition("c2m-", args.c2m_docs, world, rank)
        a, o, dd = synth.text_updates_docs(idx, args.updates)
        cm = {"arena": a, "upd_off": o, "doc_upd": dd, "n": len(idx), "n_upd": int(dd[-1]), "bytes": len(a)}
        cm["da"], cm["do"], cm["dd"] = be.put(a, 64), be.put(o.view(np.int64)), be.put(dd.view(np.int32))
        lm = np.diff(o.astype(np.int64))
        if isinstance(be, GpuBackend) and lm.max(initial=0) < 65536:   # the compact input form, as the headline
            cm["doff"] = be.put(o[dd].view(np.int64))
            cm["dlen"] = be.put(lm.astype(np.uint16).view(np.int16))
            del lm
        sm = max(args.steps // 4, 2)
        dtm, kmsm, outm, rm = time_merge(be, cm, sm, 1, dist)
        dtm = allmax(dtm, dist, dev)
        tot = allsum([cm["n"], cm["bytes"] + outm, cm["bytes"]], dist, dev)
        if rank == 0:
            pr = None
            if not args.dry_run:
                import oracle
                st, off, ln, data = be.fetch(rm, cm["n"])
                ups_of = lambda d: [a[o[u]:o[u + 1]].tobytes() for u in range(dd[d], dd[d + 1])]
                checked = 0
                for d in range(0, cm["n"], max(1, cm["n"] // 200)):
                    exp = oracle.merge_updates(ups_of(d))
                    assert exp == (int(st[d]), data[int(off[d]):int(off[d]) + int(ln[d])]), f"parity failure on c2_1m document {d}"
                    checked += 1
                assert (st == 0).all()
                pr = f"bit-exact vs oracle on {checked} sampled docs; all {cm['n']} statuses OK"
            line["c2_1m"] = {"workload": f"C2 shape at {args.c2m_docs} documents in all ('c2m-<i>' sharded by fnv1a64(name) mod {world}), "
                                         f"{args.updates} single-char insert updates each, batched Y.mergeUpdates, inputs resident in HBM",
                             "docs_total": int(tot[0]), "bytes_in_total": int(tot[2]), "steps": sm,
                             "value": round(tot[1] * sm / dtm / 1e6, 3), "unit": "MB/s", "docs_per_s": round(tot[0] * sm / dtm, 1),
                             "ms_per_step": round(dtm / sm * 1e3, 4),
                             "roofline": roof(cm["bytes"] + outm, kmsm, "k_merge_lean (rank 0)", _pmc(PMC_PROFILE, "k_merge_lean@1m")),
                             "parity": pr}
        del cm, a, o, dd
    # ---- C4: 1M merged states, state vector + diffUpdate (strong scaling over the ranks)
    if args.c4_docs:
        from tools import synth
        idx = synth.partition("c4-", args.c4_docs, world, rank)
        arena, doc_off, sva, sv_off = synth.text_states(0, seed=3, idx=idx)
        c = {"arena": arena, "doc_off": doc_off, "sva": sva, "sv_off": sv_off, "n": len(idx), "bytes": len(arena), "sv_bytes": len(sva)}
        c["da"] = be.put(arena, 64)
        c["do"] = be.put(doc_off.view(np.int64))
        c["ds"] = be.put(sva, 64)
        c["dso"] = be.put(sv_off.view(np.int64))
        blk = {"docs_total": args.c4_docs, "bytes_in_total": None, "steps": args.c4_steps,
               "workload": f"C4: {args.c4_docs} merged Y.Text states 'c4-<i>' (1-16 clients, log-uniform 1-8 KB, one state "
                           f"vector each, 10 % empty) sharded by fnv1a64(name) mod {world}, inputs resident in HBM"}
        for op in ("sv", "diff"):
            dto, kmo, ro, lean, exact = time_doc(be, c, op, args.c4_steps, dist)
            algo = c["bytes"] + int(ro.payload_bytes) + (c["sv_bytes"] if op == "diff" else 0)
            dto = allmax(dto, dist, dev)
            tot = allsum([algo, c["n"], c["bytes"]], dist, dev)
            if rank == 0:
                blk["bytes_in_total"] = int(tot[2])
                pr = None
                if not args.dry_run:
                    import oracle
                    st, off, ln, data = be.fetch(ro, c["n"])
                    checked = 0
                    for d in range(0, c["n"], max(1, c["n"] // 300)):
                        u = arena[doc_off[d]:doc_off[d + 1]].tobytes()
                        exp = oracle.encode_state_vector_from_update(u) if op == "sv" else oracle.diff_update(u, sva[sv_off[d]:sv_off[d + 1]].tobytes())
                        got = (int(st[d]), data[int(off[d]):int(off[d]) + int(ln[d])] if st[d] == 0 else None)
                        assert exp == got, f"parity failure on C4 document {d} ({op})"
                        checked += 1
                    pr = f"bit-exact vs oracle on {checked} sampled docs"
                blk[op] = {"value": round(tot[0] * args.c4_steps / dto / 1e6, 3), "unit": "MB/s",
                           "docs_per_s": round(tot[1] * args.c4_steps / dto, 1), "ms_per_step": round(dto / args.c4_steps * 1e3, 4),
                           "walker_docs_rank0": int(lean), "exact_kernel_docs_rank0": int(exact),
                           "roofline": roof(algo, kmo, f"k_doc_walk<{0 if op == 'sv' else 1}> + k_doc for deferred docs (rank 0)",
                                            _pmc(PMC_C4, f"k_doc_walk<{0 if op == 'sv' else 1}>")),
                           "parity": pr}
        if rank == 0:
            line["c4"] = blk
            if not args.dry_run and args.host_api and "host_api" in line:
                line["host_api"]["c4_diff"] = host_api_doc(be, c, "diff", min(c["n"], 250000))
        c4 = c
    # ---- f-1: doc-normalized snapshots of merged debounce logs (C2 with 20 % deletes)
    if args.f1_docs and rank == 0 and not args.dry_run:
        line["f1"] = f1_block(be, args)
    # ---- C2 past the lean envelope (multi-character inserts, up to 8 clients, deletions)
    if args.mixed and rank == 0 and not args.dry_run:
        line["c2_mixed"] = mixed_block(be, args)
    # ---- f-4: the C2 merge in update format V2
    if args.v2 and rank == 0 and not args.dry_run:
        line["v2"] = v2_block(be, args)
    # ---- C3 at full size (100 000 [snapshot, ...log] documents, 0.77 GB): one batch, rank 0 at N = 1
    if args.c3 and rank == 0 and world == 1 and not args.dry_run:
        blk = big_run(args, "c3full", be.dev.index)
        blk["roofline"] = roof(blk["bytes_in"] + blk["bytes_out"], blk["gpu_ms"], "merge cascade (k_big_scan + k_merge_big mid / 16-wave sizes + "
                               "lean / wave for the routing)", _pmc(PMC_BLOCKS, "c3full"))
        line["c3"] = blk
    # ---- C5 at BASELINE size (1 000 XmlFragment [snapshot, ...log] documents, exactly max_clients = 10 000 client blocks per snapshot,
    #      tools/synth.c): rank 0 at N = 1
    if args.c5_docs and rank == 0 and world == 1 and not args.dry_run:
        a5 = argparse.Namespace(**vars(args))
        a5.big_docs = args.c5_docs
        blk = big_run(a5, "c5", be.dev.index)
        blk["roofline"] = roof(blk["bytes_in"] + blk["bytes_out"], blk["gpu_ms"], "merge cascade (k_big_scan + k_merge_big for these documents)",
                               _pmc(PMC_BLOCKS, "c5"))
        line["c5"] = blk
    # ---- the default product store (merge + normalized snapshot) at C5 size: rank 0 at N = 1
    if args.store_docs and rank == 0 and world == 1 and not args.dry_run:
        line["c5_store"] = store_block(be, args)
    # ---- CPU baselines (rank 0 at N = 1 only)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run:
        cores = cpu_cores(args)
        from tools import synth
        idx = synth.partition("c2-", args.docs, 1, 0)
        a2, o2, d2 = synth.text_updates_docs(idx, args.updates)
        c2 = {"arena": a2, "upd_off": o2, "doc_upd": d2, "n": len(idx)}
        port = cpu_port_merge(c2, cores, args.cpu_seconds)
        y = None if args.no_yjs else cpu_yjs("merge", c2, cores, min(c2["n"], 4000))
        if y and "value" in y:
            line["cpu_baseline"] = dict(y, port=port, host=host_cpus())
        else:
            line["cpu_baseline"] = dict(port, yjs=y, host=host_cpus())
        if args.c4_docs:
            for op in ("sv", "diff"):
                e = {"port": cpu_port_doc(c4, op, cores, min(c4["n"], 200000))}
                if not args.no_yjs:
                    e["yjs"] = cpu_yjs(op, c4, cores, min(c4["n"], 60000))
                line["c4"][op]["cpu_baseline"] = e
    return line


def big_run(args, kind, dev_index=0):
    """C3 / C5 ([snapshot, ...log] large documents): the whole batch merged on the GPU
    (device-resident inputs, host-driven tier cascade, kernel time from the engine's HIP events) and
    by the CPU oracle and yjs on the host threads over the same documents."""
    import torch
    import oracle
    from hocuspocus_amd import Engine
    from tools import synth
    xml = kind == "c5"
    n = args.big_docs or (20 if xml else 100000 if kind == "c3full" else 2000)
    if xml:
        arena, upd_off, doc_upd = synth.big_docs(n, 1_000_000, 64 * 1024, max_clients=10000, max_k=50, xml=True, seed=9)
    elif kind == "c3full":   # BASELINE C3 at full size: 100 000 documents, 10 MB * rank^-0.8 (0.45 GB)
        arena, upd_off, doc_upd = synth.big_docs(n, 10_000_000, 1024, max_clients=64, max_k=200, seed=8)
    else:
        arena, upd_off, doc_upd = synth.big_docs(n, 1_000_000, 1024, max_clients=64, max_k=200, seed=8)
    dev = torch.device("cuda", dev_index)
    da = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).to(dev)
    do = torch.from_numpy(upd_off.view(np.int64)).to(dev)
    dd = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
    e = Engine(dev_index)
    runs = []
    for it in range(4):   # the first run grows the scratch; the median of the other three is reported
        s0 = e.stats()
        r = e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), n)
        s1 = e.stats()
        if it:
            runs.append(s1.kernel_ms - s0.kernel_ms)
    ms = sorted(runs)[1]
    algo = len(arena) + r.payload_bytes
    # parity: a sample of documents (all of the largest 50) against the oracle
    torch.cuda.synchronize()
    st_g = _d2h(r.status, 4 * n).view(np.int32); off_g = _d2h(r.off, 8 * n).view(np.uint64); ln_g = _d2h(r.len, 8 * n).view(np.uint64)
    ups = synth.split(arena, upd_off)
    checked = 0
    for d in sorted(set(list(range(min(n, 50))) + list(range(0, n, max(1, n // 200))))):
        exp = oracle.merge_updates(ups[doc_upd[d]:doc_upd[d + 1]])
        got = (int(st_g[d]), _d2h(r.data + int(off_g[d]), int(ln_g[d])).tobytes() if st_g[d] == 0 else None)
        assert exp == got, f"parity failure on document {d}"
        checked += 1
    cores = cpu_cores(args)
    t0 = time.perf_counter()
    st, calgo = oracle.merge_batch(arena, upd_off, doc_upd, cores)
    cdt = time.perf_counter() - t0
    assert (st == 0).all()
    sizes = np.diff(upd_off[doc_upd].astype(np.int64))
    port = {"ms": round(cdt * 1e3, 3), "MBps": round(calgo / cdt / 1e6, 1), "cores": cores, "host": host_cpus(), "kind": "port",
            "sample": "all documents of the batch through oracle/yjs_oracle.c yo_merge_batch, one pass"}
    ny = n if kind != "c5" else min(n, 200)   # C5: a bounded yjs sample (the first documents are the largest)
    y = None if (args.no_yjs or args.no_cpu_baseline) else cpu_yjs("merge", {"arena": arena, "upd_off": upd_off, "doc_upd": doc_upd}, cores, ny)
    if y and "value" in y:
        y["ms"] = round(n / y["docs_per_s"] * 1e3, 3)   # the whole batch (slowest worker)
        if ny < n:
            y["ms_note"] = f"extrapolated from the first {ny} documents' rate (the largest ones) to all {n}"
    # the same batch through the host API (ygm_merge_v1: 64 MB chunks of documents over the stage contexts, pinned
    # staging, PCIe both ways): the production call, where the large-document tier's second stream shares the process's
    # hardware queues with the stage streams
    upd_doc = np.repeat(np.arange(n, dtype=np.uint32), np.diff(doc_upd.astype(np.int64)))
    e.merge_packed_raw(arena, upd_off, upd_doc, n)   # (warm-up: stage contexts, pinned buffers)
    h0 = _host_stats(e)
    t0 = time.perf_counter()
    hreps = 2
    for _ in range(hreps):
        hst, hoff, hln, hdata = e.merge_packed_raw(arena, upd_off, upd_doc, n)
    hwall = (time.perf_counter() - t0) / hreps
    h1 = _host_stats(e)
    hd = {k: (h1[k] - h0[k]) / hreps for k in h0}
    for d in list(range(min(n, 5))) + [n - 1]:   # (the largest documents and the last)
        got = (int(hst[d]), bytes(hdata[int(hoff[d]):int(hoff[d]) + int(hln[d])]) if hst[d] == 0 else None)
        assert oracle.merge_updates(ups[doc_upd[d]:doc_upd[d + 1]]) == got, f"host API parity failure on document {d}"
    host = {"op": "merge (ygm_merge_v1, host arrays)", "wall_ms": round(hwall * 1e3, 3),
            "value": round((len(arena) + int(hln.sum())) / hwall / 1e6, 1), "unit": "MB/s end-to-end (PCIe + host staging included)",
            "h2d_ms": round(hd["h2d_ms"], 3), "d2h_ms": round(hd["d2h_ms"], 3), "device_span_ms": round(hd["kernel_ms"], 3),
            "parity": "bit-exact vs oracle on the 5 largest documents and the last"}
    e.close()
    return {"config": kind.upper(), "op": "merge", "docs": n, "bytes_in": len(arena), "bytes_out": int(r.payload_bytes), "host_api": host,
            "largest_doc": int(sizes.max()),
                      "gpu_ms": round(ms, 3), "gpu_runs_ms": [round(x, 3) for x in runs], "gpu_MBps": round(algo / ms / 1e3, 1), "gpu_docs_per_s": round(n / ms * 1e3),
                      "docs_big_tier": s1.docs_big - s0.docs_big, "docs_seq_tier": s1.docs_seq - s0.docs_seq,
                      "parity": f"bit-exact vs oracle on {checked} documents (the 50 largest + an even sample)",
                      "cpu_baseline": dict(port, yjs=y)}


def big_line(args):
    print(json.dumps(big_run(args, args.big)), flush=True)


def block_line(args):
    """One side block alone (rank 0, N = 1): the command the block's PMC passes profile."""
    be = GpuBackend(0)
    fn = {"f1": f1_block, "mixed": mixed_block, "v2": v2_block, "store": store_block}[args.block]
    print(json.dumps(fn(be, args)), flush=True)
    be.close()


def main():
    args = parse()
    if args.big:
        return big_line(args)
    if args.block:
        return block_line(args)
    in_torchrun = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not in_torchrun:
        sys.exit(spawn_ranks(args))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if in_torchrun:
        assert world == args.gpus, f"WORLD_SIZE {world} != --gpus {args.gpus}"
    dist, dev = None, None
    if args.dry_run:
        be = DryBackend()
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
    else:
        import torch
        be = GpuBackend(local)
        dev = be.dev
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    line = run_rank(args, rank, world, dist, be, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    be.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
