"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (measurement tooling): per-dispatch averages
and derived ratios.  python tools/sq_summary.py <rocprof out dir>"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if k.startswith("__amd"):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, d in acc.items():
    n = len(disp[k])
    a = {c: v / n for c, v in d.items()}
    w = a.get("SQ_WAVES", 0) or 1
    print(f"{k}: {n} dispatches")
    for c in sorted(a):
        print(f"  {c:24s} {a[c]:14.4g}   per wave {a[c] / w:12.4g}")
    if "SQ_WAVE_CYCLES" in a:
        wc = a["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in a:
                print(f"  {c} / WAVE_CYCLES = {a[c] / wc:.3f}")
