"""HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of the same command, with the
launches of one kernel split by workload (tooling).  A bench run launches one kernel on several workloads (the
headline C2 batch, c2_100k, c2_1m ...): launches are told apart by their duration, which differs by an order of
magnitude between the workloads.  FETCH_SIZE is doubled (gfx950 wide-read undercount, MI355X_MICROARCH.md HBM
section), both counters are KiB.

    python tools/pmc_split.py <fetch dir> <write dir> <out.json> KERNEL:LABEL:MIN_US:MAX_US ...

e.g. k_merge_lean<0>:k_merge_lean@10k:20:100  k_merge_lean<0>:k_merge_lean@100k:200:800"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    out = {}
    for p in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            if r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ygm::", "")
            disp = r["Dispatch_Id"]
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            e = out.setdefault((k, disp), [0.0, us])
            e[0] += float(r["Counter_Value"])
    return out


def main():
    fd, wd, outp = sys.argv[1:4]
    f = per_dispatch(fd, "FETCH_SIZE")
    w = per_dispatch(wd, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes of the same command), per dispatch, "
                     "launches of a kernel split by workload (duration range)",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount, MI355X_MICROARCH.md HBM section)", "kernels": {}}
    for spec in sys.argv[4:]:
        kern, label, lo, hi = spec.split(":")
        lo, hi = float(lo), float(hi)
        fs = [v[0] for (k, _), v in f.items() if k == kern and lo <= v[1] <= hi]
        ws = [v[0] for (k, _), v in w.items() if k == kern and lo <= v[1] <= hi]
        if not fs or not ws:
            print(f"{label}: no launches of {kern} in [{lo}, {hi}] us", file=sys.stderr)
            continue
        rd = sum(fs) / len(fs) * 1024 * 2
        wr = sum(ws) / len(ws) * 1024
        res["kernels"][label] = {"kernel": kern, "launches": [len(fs), len(ws)], "fetch_bytes": rd, "write_bytes": wr,
                                 "hbm_bytes_per_launch": rd + wr}
        res[label] = rd + wr
    if "k_merge_lean@10k" in res:
        res["hbm_bytes_per_launch"] = res["k_merge_lean@10k"]
    json.dump(res, open(outp, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
