"""Print the last frame's kernel timeline from a rocprofv3 kernel-trace database: start offset,
duration and queue (stream) of every dispatch, so overlapped streams can be read side by side.

Usage: python tools/timeline.py run_results.db [dispatches]   (default: the last 40)"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    # the runtime's own copy / fill kernels after the timed frames (readbacks) are left out
    rows = [r for r in db.cursor().execute("select name, start, end, queue_id from kernels order by start")
            if not r[0].startswith("__amd_rocclr_copyBuffer")][-n:]
    t0 = rows[0][1]
    queues = sorted({r[3] for r in rows})
    for name, s, e, q in rows:
        short = name.replace("vx::(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:28]
        col = queues.index(q)
        print("%9.1f %7.1f  %s%-28s" % ((s - t0) / 1e3, (e - s) / 1e3, " " * 30 * col, short))
    span = (rows[-1][2] - t0) / 1e3
    busy = 0.0
    ivs = sorted((s, e) for _, s, e, _ in rows)
    cs, ce = ivs[0]
    for s, e in ivs[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print("span %.1f us, some kernel running %.1f us (%.0f %%)" % (span, busy / 1e3, 100.0 * busy / 1e3 / span))


if __name__ == "__main__":
    main()
