"""Per-kernel sums of a rocprofv3 --pmc counter_collection.csv, divided by SQ_WAVES (tooling).

    python tools/sq_summary.py <counter_collection.csv>"""
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set); dur = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("ygm::", "")[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r["Dispatch_Id"])
    dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in sorted(agg.items(), key=lambda x: -sum(dur[x[0]].values())):
    t = sum(dur[k].values())
    if t < 500: continue
    w = v.get("SQ_WAVES", 0) or 1
    s = " ".join(f"{c.replace('SQ_','')}={v[c]/w:.0f}" for c in sorted(v) if c != "SQ_WAVES")
    print(f"{k:60s} n={len(cnt[k])} ms={t/1e3:.2f} waves={w:.0f} per-wave: {s}")
