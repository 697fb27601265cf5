"""Per-kernel HBM traffic from two separate rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), corrected as /opt/skills/guides/MI355X_MICROARCH.md
§HBM prescribes for gfx950:
  * both counters are in KiB (rocprofv3 derived-counter expressions /1024);
  * FETCH_SIZE reports 1/2 of the bytes of wide coalesced streaming reads
    -> doubled;  WRITE_SIZE is exact for 16-B/lane stores and float atomics.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json
(each DIR holds run_counter_collection.csv of one pass over the same workload)
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "")
    n = n.split("(")[0]
    n = re.sub(r"^lsr::", "", n)
    return n


def per_dispatch(path: str, counter: str) -> dict:
    """{kernel: [value per dispatch]} (rows of one dispatch are summed)."""
    acc = defaultdict(float)
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            d = int(row["Dispatch_Id"])
            acc[d] += float(row["Counter_Value"])
            names[d] = short(row["Kernel_Name"])
    out = defaultdict(list)
    for d in sorted(acc):
        out[names[d]].append(acc[d])
    return out


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch = per_dispatch(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE")
    write = per_dispatch(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        fv, wv = fetch.get(k, []), write.get(k, [])
        f_kib = sum(fv) / len(fv) if fv else 0.0
        w_kib = sum(wv) / len(wv) if wv else 0.0
        res[k] = {
            "dispatches": max(len(fv), len(wv)),
            "fetch_kib_raw": round(f_kib, 1),
            "write_kib_raw": round(w_kib, 1),
            "fetch_bytes": int(2 * f_kib * 1024),
            "write_bytes": int(w_kib * 1024),
            "traffic_bytes": int(2 * f_kib * 1024 + w_kib * 1024),
        }
    doc = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; KiB->bytes; "
                     "FETCH doubled (gfx950 wide-read correction, MI355X_MICROARCH.md §HBM)",
           "kernels": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes"]):
        print(f"{k:60s} n={v['dispatches']:4d} fetch={v['fetch_bytes'] / 1e6:9.2f} MB "
              f"write={v['write_bytes'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
