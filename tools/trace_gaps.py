"""Kernel durations and inter-dispatch gaps from a rocprofv3 kernel_trace.csv (tooling)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/*kernel_trace.csv")[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
prev_end = None
tail = rows[-int(sys.argv[2]) if len(sys.argv) > 2 else -12:]
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1000 if prev_end else 0
    print(f"{r['Kernel_Name'][:40]:40s} dur {(e - s) / 1000:8.2f} us  gap-before {gap:8.2f} us")
    prev_end = e
