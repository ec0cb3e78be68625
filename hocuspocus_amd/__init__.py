"""MI355X-native batched Yjs update engine for Hocuspocus's persistence / sync hot path.

The product is ``libygm.so`` (HIP kernels for gfx950 + C-ABI runtime,
``include/ygm.h``); :mod:`hocuspocus_amd.engine` is its Python binding and
:mod:`hocuspocus_amd.shard` routes documents over a node's GPUs.  The Hocuspocus
Extension / DocumentStore drop-in (packages/server/src/types.ts:36-63,
packages/extension-database/src/Database.ts:10-60) is the Node package
``packages/extension-gpu-merge`` over the same C ABI (N-API addon).
"""
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))


def build(arch: str = "gfx950") -> str:
    """Compiles libygm.so in-tree with hipcc (cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(_HERE, "csrc"), f"ARCH={arch}"])
    return os.path.join(_HERE, "libygm.so")


from .engine import Engine, YjsError, DeviceResult  # noqa: E402,F401
