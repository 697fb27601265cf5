"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd .db) into a
markdown table under profiles/.  Usage: python tools/prof_summary.py DB OUT.md [title]"""
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else db
    cur = sqlite3.connect(db).cursor()
    rows = list(cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats: {title}\n\n")
        f.write("| kernel | calls | total us | avg us | % |\n|---|---|---|---|---|\n")
        for name, calls, tot, avg, pct in rows:
            short = name.split("(")[0].replace("void ", "")
            f.write(f"| `{short}` | {calls} | {tot:.1f} | {avg:.1f} | {pct:.2f} |\n")
    print(open(out).read())


if __name__ == "__main__":
    main()
