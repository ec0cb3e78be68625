"""Kernel-time probe for merge builds (tooling): C2 inputs resident on cuda:0, N device merges,
mean HIP-event kernel ms.  Used with YGM_LIB=<experiment .so> (e.g. phase-stop builds)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hocuspocus_amd import Engine  # noqa: E402
from tools import synth  # noqa: E402

arena, upd_off, doc_upd = synth.text_updates(10000, 200, seed=1000)
dev = torch.device("cuda", 0)
da = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).to(dev)
do = torch.from_numpy(upd_off.view(np.int64)).to(dev)
dd = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
e = Engine(0)
for _ in range(3):
    e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), 10000)
s0 = e.stats()
n = 20
for _ in range(n):
    e.merge_device(da.data_ptr(), len(arena), do.data_ptr(), dd.data_ptr(), int(doc_upd[-1]), 10000)
s1 = e.stats()
print(os.environ.get("YGM_LIB", "libygm.so"), "lean kernel ms", round((s1.lean_ms - s0.lean_ms) / n, 4),
      "total kernel ms", round((s1.kernel_ms - s0.kernel_ms) / n, 4))
