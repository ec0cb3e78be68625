"""Lane-iteration census of the SV / diff ring walker on C4 (diagnostic build libygm_diag.so; tooling).
Counts: fast-decoder units, general-decoder units, lanes waiting for ring data, idle / finishing /
state-vector lanes, long-string continuation; rounds; wave-iterations that ran the general decoder;
and the wave shader-clock split over the round's sections."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hocuspocus_amd.engine as eng  # noqa: E402

eng.LIB_PATH = os.path.join(ROOT, "hocuspocus_amd", "libygm_diag.so")
from tools import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
arena, doc_off, sva, sv_off = synth.text_states(n, seed=3)
dev = torch.device("cuda", 0)
da = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).to(dev)
do = torch.from_numpy(doc_off.view(np.int64)).to(dev)
ds = torch.from_numpy(np.concatenate([sva, np.zeros(64, np.uint8)])).to(dev)
dso = torch.from_numpy(sv_off.view(np.int64)).to(dev)
e = eng.Engine(0)
L = eng.lib()
L.ygm_walk_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(16, np.uint64)
names = ["fast", "general", "not_ready", "idle", "string", "rounds", "general_iters", "fast_items"]
for op in ("sv", "diff"):
    L.ygm_walk_diag_read(buf.ctypes.data, 1)
    s0 = e.stats()
    if op == "sv":
        e.sv_device(da.data_ptr(), len(arena), do.data_ptr(), n)
    else:
        e.diff_device(da.data_ptr(), len(arena), do.data_ptr(), ds.data_ptr(), dso.data_ptr(), n)
    s1 = e.stats()
    L.ygm_walk_diag_read(buf.ctypes.data, 1)
    c = {k: int(v) for k, v in zip(names, buf[0:8])}
    tot = sum(c[k] for k in names[:5])
    print(json.dumps({"op": op, "docs": n, "kernel_ms": round(s1.kernel_ms - s0.kernel_ms, 3), **c,
                      "lane_iters": tot, "frac": {k: round(c[k] / max(tot, 1), 3) for k in names[:5]},
                      "general_iter_frac": round(c["general_iters"] / max(c["rounds"] * 8, 1), 3),
                      "items_per_fast_lane_iter": round(c["fast_items"] / max(c["fast"], 1), 3),
                      "clock_frac": {k: round(int(v) / max(int(buf[8:13].sum()), 1), 3) for k, v in
                                     zip(["commit", "sv_parse", "grab_out_init", "staging", "parse"], buf[8:13])}}))
