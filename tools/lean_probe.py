"""Lean-merge probe for profiler passes and A/B builds (tooling): the c2_1m block's corpus (C2 shape, 'c2m-<i>'
documents, compact input form) merged on cuda:0 by the library named by YGM_LIB (default hocuspocus_amd/libygm.so),
best kernel time of `reps` launches, plus a digest of every document's status and bytes so variants can be
compared with the parity-tested build.

    python tools/lean_probe.py [n_docs] [reps]"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from bench import _d2h
    from hocuspocus_amd import Engine
    from tools import synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    idx = synth.partition("c2m-", n, 1, 0)
    a, o, dd = synth.text_updates_docs(idx, 200)
    dev = torch.device("cuda", 0)

    def put(x, pad=0):
        x = np.ascontiguousarray(x)
        if pad:
            x = np.concatenate([x.view(np.uint8).reshape(-1), np.zeros(pad, np.uint8)])
        return torch.from_numpy(x).to(dev)
    da = put(a, 64)
    dd_ = put(dd.view(np.int32))
    doff = put(o[dd].view(np.int64))
    dlen = put(np.diff(o.astype(np.int64)).astype(np.uint16).view(np.int16))
    e = Engine(0)
    s = torch.cuda.current_stream(dev).cuda_stream
    best, r = None, None
    for _ in range(reps):
        s0 = e.stats()
        e.merge_device_lens_async(da, len(a), doff, dlen, dd_, int(dd[-1]), n, s)
        r = e.merge_device_finish()
        s1 = e.stats()
        ms = s1.kernel_ms - s0.kernel_ms
        best = ms if best is None or ms < best else best
    torch.cuda.synchronize()
    st = _d2h(r.status, n * 4).view(np.int32)
    off = _d2h(r.off, n * 8).view(np.uint64)
    ln = _d2h(r.len, n * 8).view(np.uint64)
    data = _d2h(r.data, int(r.data_bytes))
    h = hashlib.sha256(st.tobytes())
    h.update(ln.tobytes())
    # bytes in document order (slot offsets may differ between variants): one gather
    idxs = np.concatenate([np.arange(int(off[d]), int(off[d] + ln[d])) for d in range(0, n, max(1, n // 20000))])
    h.update(data[idxs].tobytes())
    algo = len(a) + int(r.payload_bytes)
    print(json.dumps({"lib": os.path.basename(os.environ.get("YGM_LIB", "libygm.so")), "docs": n, "best_ms": round(best, 4),
                      "frac": round(algo / best / 1e6 / 8000.0, 4), "docs_lean": s1.docs_lean - s0.docs_lean,
                      "digest": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
