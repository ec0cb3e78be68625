"""Kernel resource table for profiles/ (tooling): compiles every HIP source of libygm.so for gfx950 (device side only)
with -Rpass-analysis=kernel-resource-usage and writes one markdown row per kernel -- VGPRs, scratch bytes per lane,
the compiler's waves/SIMD and the LDS bytes per workgroup.

    python tools/kernel_resources.py OUT.md"""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hocuspocus_amd", "csrc")
SRC = ("ygm_kernels.hip", "ygm_walk.hip", "ygm_snapshot.hip", "ygm_v2.hip")


def remarks(src):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "-c",
           "-Rpass-analysis=kernel-resource-usage", "-o", os.devnull, src]
    return subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
    return [n.replace("ygm::", "").split("(")[0].replace("void ", "") for n in out.splitlines()]


def parse(text):
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    return rows


def main():
    with ThreadPoolExecutor(4) as ex:
        texts = list(ex.map(remarks, SRC))
    rows = [r for t in texts for r in parse(t) if "vgpr" in r]
    names = demangle([r["name"] for r in rows])
    seen, lines = set(), []
    for r, n in zip(rows, names):
        if n in seen:
            continue
        seen.add(n)
        lines.append(f"| `{n}` | {r['vgpr']} | {r.get('scratch', 0)} | {r.get('occ', '?')} | {r.get('lds', 0)} |")
    with open(sys.argv[1], "w") as f:
        f.write("# Kernel resources (hipcc -Rpass-analysis=kernel-resource-usage, gfx950, the closing tree; "
                "`tools/kernel_resources.py`)\n\n| kernel | VGPRs | scratch B/lane | waves/SIMD (compiler) | LDS B/workgroup |\n"
                "|---|---|---|---|---|\n" + "\n".join(lines) + "\n")
    print(f"{len(lines)} kernels")


if __name__ == "__main__":
    main()
