"""Per-launch durations (ms) of the ygm kernels in a rocprofv3 --kernel-trace csv directory (tooling).

    python tools/ktrace.py <dir> [substring]"""
import collections
import csv
import glob
import os
import sys

d = collections.defaultdict(list)
for p in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ygm::", "")
        if len(sys.argv) < 3 or sys.argv[2] in k:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    print(k[:60], [round(x, 2) for x in v])
