"""Per-kernel duration summary from a rocprofv3 rocpd database (run_results.db):
python tools/rocpd_stats.py DB [N]  -> name, calls, median / min / mean us, sorted by total."""
import collections
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = sqlite3.connect(db)
q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
agg = collections.defaultdict(list)
for n, s, e in c.execute(q):
    agg[n].append(e - s)
print(f"{'kernel':60s} {'calls':>5s} {'med us':>9s} {'min us':>9s} {'mean us':>9s}")
for n, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:top]:
    v = sorted(v)
    print(f"{n[:60]:60s} {len(v):5d} {v[len(v) // 2] / 1e3:9.1f} {v[0] / 1e3:9.1f} {sum(v) / len(v) / 1e3:9.1f}")
