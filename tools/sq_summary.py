"""Per-kernel mean of every PMC counter in rocprofv3 counter_collection CSVs (tooling)."""
import collections
import csv
import glob
import sys

for path in sys.argv[1:]:
    for f in glob.glob(path + "/*counter_collection.csv"):
        rows = list(csv.DictReader(open(f)))
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in rows:
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in agg.items():
            if "rocclr" in k:
                continue
            print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
