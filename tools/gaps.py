"""Idle gaps between consecutive kernels of the timed steps in a rocprofv3
--kernel-trace CSV: per kernel name, the median gap before its dispatch."""
import csv
import statistics
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
rows.sort()
gaps = defaultdict(list)
prev_end = None
for s, e, n in rows:
    if prev_end is not None:
        gaps[n].append((s - prev_end) / 1000.0)
    prev_end = max(prev_end or 0, e)
tot = 0.0
for n, g in sorted(gaps.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    m = statistics.median(g)
    print(f"{n:60s} n={len(g):4d} median gap before {m:8.2f} us")
