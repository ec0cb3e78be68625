"""SQ counters per dispatch of one kernel (tooling): python tools/sq_dispatch.py <pmc dir> <kernel name substring>"""
import csv, glob, os, sys, collections
d = sys.argv[1]; kern = sys.argv[2]
acc = collections.defaultdict(list)
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if kern not in k: continue
        acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
        acc[(r["Dispatch_Id"], "_us")] = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3]
disp = sorted({k[0] for k in acc}, key=int)
for dd in disp:
    row = {c: sum(v) for (x, c), v in acc.items() if x == dd}
    print(dd, {k: (round(v) if v > 100 else round(v, 2)) for k, v in sorted(row.items())})
