"""Host vs GPU timeline of each forward's binning in a rocprofv3 kernel + HIP API
trace (csv): for each k_bin_count dispatch, the times (us, relative to the
count's end) of the HIP calls between the count's launch and the scatter's
launch, and of the table / apply / scatter kernels.  Usage: host_timeline.py DIR"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
K = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
A = list(csv.DictReader(open(glob.glob(os.path.join(d, "*hip_api_trace.csv"))[0])))
api = {int(r["Correlation_Id"]): r for r in A}
A.sort(key=lambda r: int(r["Start_Timestamp"]))
K.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    for k in ("k_bin_count", "k_bin_table", "k_tile_start_apply", "k_bin_scatter", "k_tile_sort_wave",
              "k_preprocess_colour", "k_preprocess<", "k_render_fwd", "k_render_bwd"):
        if k in n:
            return k
    return n[:30]


rel = {}
for i, k in enumerate(K):
    if short(k["Kernel_Name"]) != "k_bin_count":
        continue
    ce = int(k["End_Timestamp"])
    c0 = api[int(k["Correlation_Id"])]
    nxt = {}
    for k2 in K[i + 1:i + 6]:
        nxt.setdefault(short(k2["Kernel_Name"]), k2)
    if "k_bin_scatter" not in nxt:
        continue
    s = nxt["k_bin_scatter"]
    s_api = api[int(s["Correlation_Id"])]
    # host calls from the count's launch to the scatter's launch (same thread)
    t0, t1 = int(c0["Start_Timestamp"]), int(s_api["End_Timestamp"])
    calls = [r for r in A if t0 <= int(r["Start_Timestamp"]) <= t1 and r["Thread_Id"] == c0["Thread_Id"]]
    for j, r in enumerate(calls):
        key = f"{j:02d} {r['Function']}"
        rel.setdefault(key + " start", []).append((int(r["Start_Timestamp"]) - ce) / 1e3)
        rel.setdefault(key + " end", []).append((int(r["End_Timestamp"]) - ce) / 1e3)
    for n in ("k_bin_table", "k_tile_start_apply", "k_bin_scatter"):
        if n in nxt:
            rel.setdefault("GPU " + n + " start", []).append((int(nxt[n]["Start_Timestamp"]) - ce) / 1e3)
            rel.setdefault("GPU " + n + " end", []).append((int(nxt[n]["End_Timestamp"]) - ce) / 1e3)
    rel.setdefault("GPU k_bin_count start", []).append((int(k["Start_Timestamp"]) - ce) / 1e3)
rows = sorted(((statistics.median(v), k, len(v)) for k, v in rel.items()))
for m, k, n in rows:
    print(f"{m:9.2f} us  {k}  (n={n})")

# the scatter's own launch call per forward
print("scatter launch call (start, end) and kernel start, us after the count's end:")
for i, k in enumerate(K):
    if short(k["Kernel_Name"]) != "k_bin_count":
        continue
    ce = int(k["End_Timestamp"])
    for k2 in K[i + 1:i + 6]:
        if short(k2["Kernel_Name"]) == "k_bin_scatter":
            a = api[int(k2["Correlation_Id"])]
            print(f"  {(int(a['Start_Timestamp']) - ce) / 1e3:8.2f} {(int(a['End_Timestamp']) - ce) / 1e3:8.2f}"
                  f"  kernel {(int(k2['Start_Timestamp']) - ce) / 1e3:8.2f}")
            break
