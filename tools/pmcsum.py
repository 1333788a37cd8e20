"""Per-kernel PMC summary from rocprofv3 DBs: python tools/pmcsum.py DB [DB...]
Prints, per kernel name, the mean over dispatches of each counter (last dispatches of the run)."""
import collections
import sqlite3
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    cur = sqlite3.connect(path).cursor()
    for name, cnt, val, disp, grid in cur.execute(
            "select kernel_name, counter_name, value, dispatch_id, grid_size from counters_collection"):
        n = name.replace("vx::(anonymous namespace)::", "").split("(")[0]
        agg[(n, grid)][cnt].append(val)
for (k, grid), d in sorted(agg.items()):
    parts = ["%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(d.items())]
    print("%-22s grid=%-9d n=%-3d %s" % (k, grid, len(next(iter(d.values()))), " ".join(parts)))
