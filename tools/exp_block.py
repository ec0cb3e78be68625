"""One bench.py block alone (tooling): v2 (C2 converted to V2, ygm_merge_v2_device per step), mixed (c2_mixed through
the tier cascade) or f1 (doc-normalized snapshots), each with its parity sample and without CPU baselines.
    python tools/exp_block.py [docs] [block]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    block = sys.argv[2] if len(sys.argv) > 2 else "v2"
    be = bench.GpuBackend(0)
    args = argparse.Namespace(docs=n, updates=200, no_cpu_baseline=True, no_yjs=True, f1_docs=n, cpu_threads=0)
    fn = {"v2": bench.v2_block, "mixed": bench.mixed_block, "f1": bench.f1_block}[block]
    print(json.dumps({"block": block, **fn(be, args)}), flush=True)
    be.close()


if __name__ == "__main__":
    main()
