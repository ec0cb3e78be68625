"""V2 merge step timing (tooling): bench.py's v2 block alone (C2 converted to V2, ygm_merge_v2_device per step,
parity on a sample), without its CPU baseline.
    python tools/exp_v2.py [docs]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    be = bench.GpuBackend(0)
    args = argparse.Namespace(docs=n, updates=200, no_cpu_baseline=True, no_yjs=True)
    print(json.dumps(bench.v2_block(be, args)), flush=True)
    be.close()


if __name__ == "__main__":
    main()
