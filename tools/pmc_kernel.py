"""Per-dispatch averages of every PMC counter in a rocprofv3 --pmc run, for
kernels whose name contains a substring.
Usage: python tools/pmc_kernel.py DIR SUBSTRING [DIR SUBSTRING ...]"""
import csv
import sys
from collections import defaultdict


def load(d, sub):
    acc = defaultdict(lambda: defaultdict(float))
    with open(f"{d}/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            if sub not in row["Kernel_Name"]:
                continue
            acc[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    n = len(acc)
    tot = defaultdict(float)
    for v in acc.values():
        for k, x in v.items():
            tot[k] += x
    return n, {k: x / max(n, 1) for k, x in tot.items()}


if __name__ == "__main__":
    a = sys.argv[1:]
    for d, sub in zip(a[::2], a[1::2]):
        n, c = load(d, sub)
        print(f"{d} [{sub}] dispatches={n}")
        for k in sorted(c):
            print(f"   {k:32s} {c[k]:16.0f}")
