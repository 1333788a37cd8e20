"""Host enqueue against GPU execution in a rocprofv3 --hip-trace --kernel-trace database: per HIP API
call name, count / total / max host time over the last N ms of the run; and per kernel dispatch, the
lead of its launch call's end over the kernel's start (negative: the GPU waited for the host).
python tools/api_lead.py DB [LAST_MS]"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    ks = db.execute("select name, start, end, corr_id, stream from kernels order by start").fetchall()
    t1 = ks[-1][2]
    t0 = t1 - last_ms * 1e6
    regs = db.execute("select name, start, end, corr_id from regions where start >= ? order by start", (t0,)).fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for n, s, e, _ in regs:
        a = agg[n]
        a[0] += 1
        a[1] += (e - s) / 1e3
        a[2] = max(a[2], (e - s) / 1e3)
    print("HIP API calls in the last %.1f ms (count, total us, max us):" % last_ms)
    for n, (c, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print("  %-40s %5d %10.1f %8.1f" % (n[:40], c, tot, mx))
    by_corr = {c: (s, e) for n, s, e, c in regs}
    leads = []
    for n, s, e, c, st in ks:
        if s < t0 or c not in by_corr:
            continue
        leads.append(((s - by_corr[c][1]) / 1e3, n.split("(")[0][-40:], st))
    leads.sort()
    print("kernel start - its launch call's end, us (smallest 15):")
    for l, n, st in leads[:15]:
        print("  %8.1f  %-40s %s" % (l, n, st))
    if leads:
        print("median lead %.1f us over %d dispatches" % (leads[len(leads) // 2][0], len(leads)))


if __name__ == "__main__":
    main()
