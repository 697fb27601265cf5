"""Per-step kernel timeline from a rocprofv3 --kernel-trace run (rocpd .db):
prints each kernel of one steady-state step with its duration and the idle gap
before it, plus the step span vs the summed kernel time.
Usage: python tools/timeline.py DB [first_kernel_of_step] [step_index]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_preprocess<"
    idx = int(sys.argv[3]) if len(sys.argv) > 3 else -3
    cur = sqlite3.connect(db).cursor()
    rows = list(cur.execute("select name, start, end from kernels order by start"))
    starts = [i for i, r in enumerate(rows) if first in r[0]]
    if len(starts) < 3:
        print(f"found {len(starts)} steps starting with {first!r}")
        return
    a = starts[idx]
    b = starts[idx + 1]
    t0 = rows[a][1]
    busy = 0.0
    prev_end = None
    for name, s, e in rows[a:b]:
        short = name.split("(")[0].replace("void ", "")[:60]
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        busy += (e - s) / 1e3
        print(f"{short:60s} start {(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}  gap {gap:6.1f}")
        prev_end = e
    span = (rows[b][1] - t0) / 1e3
    print(f"step span {span:.1f} us, kernel busy {busy:.1f} us, idle {span - busy:.1f} us")


if __name__ == "__main__":
    main()
