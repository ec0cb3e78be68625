"""HBM bytes per step of a whole bench block (tooling): two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of one
`bench.py --big ...` command, every ygm kernel dispatch summed (the block's cascade: scan, lean, wave, large-document
sizes ...) and divided by the command's merge calls (warm-up + timed runs).  FETCH_SIZE x2 (gfx950 wide-read
undercount, MI355X_MICROARCH.md HBM section), both counters KiB.  Merges the result into OUT under LABEL.

    python tools/pmc_blocks.py <fetch dir> <write dir> <out.json> LABEL CALLS [PREFIX,...]

PREFIX: count only the kernels whose names start with one of these (a block whose setup runs other kernels: f1's
snapshot kernels after the merge that makes its input)."""
import csv
import glob
import json
import os
import sys


def total(d, counter, prefixes=None):
    s, kern = 0.0, {}
    for p in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            if r.get("Counter_Name") != counter or "ygm" not in r["Kernel_Name"] and not r["Kernel_Name"].startswith("k_"):
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ygm::", "")
            if prefixes and not any(k.startswith(p) for p in prefixes):
                continue
            v = float(r["Counter_Value"])
            s += v
            kern[k] = kern.get(k, 0.0) + v
    return s, kern


def main():
    fd, wd, outp, label, calls = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5])
    pre = sys.argv[6].split(",") if len(sys.argv) > 6 else None
    f, fk = total(fd, "FETCH_SIZE", pre)
    w, wk = total(wd, "WRITE_SIZE", pre)
    res = json.load(open(outp)) if os.path.exists(outp) else {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes of the same bench.py --big command), every "
                  "ygm kernel dispatch summed and divided by the command's merge calls",
        "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount, MI355X_MICROARCH.md HBM section)", "blocks": {}}
    res["blocks"][label] = {"calls": calls, "fetch_bytes": f * 1024 * 2 / calls, "write_bytes": w * 1024 / calls,
                            "hbm_bytes_per_step": (f * 2 + w) * 1024 / calls,
                            "per_kernel_bytes_per_step": {k: (fk.get(k, 0) * 2 + wk.get(k, 0)) * 1024 / calls for k in sorted(set(fk) | set(wk))}}
    res[label] = res["blocks"][label]["hbm_bytes_per_step"]
    json.dump(res, open(outp, "w"), indent=1)
    print(json.dumps(res["blocks"][label], indent=1))


if __name__ == "__main__":
    main()
