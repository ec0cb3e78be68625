"""Walker HBM split (tooling): FETCH_SIZE / WRITE_SIZE per k_doc_walk launch from rocprofv3 --pmc passes named
gpurun_out/pmc_f_<tag> / pmc_w_<tag> (tools/gpu.sh `pmc`), FETCH_SIZE doubled (MI355X_MICROARCH.md HBM section),
KiB -> bytes.  Prints one JSON object {tag: {kernel: {"fetch_GB": [...], "write_GB": [...], "us": [...]}}}.

    python tools/pmc_walk.py tag [tag ...]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d, counter):
    out = collections.defaultdict(list)
    for p in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ygm::", "")
            if "walk" not in k:
                continue
            out[k].append((float(r["Counter_Value"]) * 1024, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out


res = {}
for tag in sys.argv[1:]:
    t = res.setdefault(tag, {})
    for ctr, pre, mul in (("FETCH_SIZE", "f", 2), ("WRITE_SIZE", "w", 1)):
        d = os.path.join(ROOT, "gpurun_out", f"pmc_{pre}_{tag}")
        if not os.path.isdir(d):
            continue
        for k, v in load(d, ctr).items():
            e = t.setdefault(k, {})
            e[f"{'fetch' if pre == 'f' else 'write'}_GB"] = [round(x * mul / 1e9, 3) for x, _ in v]
            e[f"us_{pre}"] = [round(u) for _, u in v]
print(json.dumps(res, indent=1))
