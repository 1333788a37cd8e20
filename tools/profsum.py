"""Summarise a rocprofv3 run_results.db: per-kernel totals and the last frame's launch sequence."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
print("%-40s %6s %10s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "pct"))
for r in cur.execute("select * from top_kernels"):
    name = r[0].replace("vx::(anonymous namespace)::", "").split("(")[0]
    # top_kernels durations are in microseconds
    print("%-40s %6d %10.3f %10.2f %6.2f" % (name[:40], r[1], r[2] / 1e3, r[3], r[4]))
if len(sys.argv) > 2:
    rows = list(cur.execute("select name, duration from kernels order by start"))
    for n, d in rows[-int(sys.argv[2]):]:
        print("  %-30s %8.1f us" % (n.replace("vx::(anonymous namespace)::", "").split("(")[0][:30], d / 1e3))
