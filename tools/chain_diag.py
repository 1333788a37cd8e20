"""Per chain kernel of the last frames: kernel-trace duration, shader clock from the PMC pass's
GRBM_GUI_ACTIVE cycles over that pass's dispatch duration, UTCL1 translation miss rate -- for the
pipelined (pipe) and frame-by-frame (calls) loops.  python tools/chain_diag.py gpurun_out/TAG"""
import collections
import sqlite3
import sys

CHAIN = ("k_firefly", "k_temporal", "k_history_fix", "k_history_clamp", "k_atrous_smem", "k_atrous_tile", "k_atrous")


def short(n):
    return n.replace("vx::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def kt(path, last=40):
    cur = sqlite3.connect(path).cursor()
    rows = list(cur.execute("select name, start, end from kernels order by start"))
    d = collections.defaultdict(list)
    for n, s, e in rows:
        k = short(n)
        if k.split("<")[0] in CHAIN:
            d[k].append((e - s) / 1e3)
    return {k: sum(v[-6:]) / len(v[-6:]) for k, v in d.items()}


def pmc(path):
    cur = sqlite3.connect(path).cursor()
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for n, c, v, disp, s, e in cur.execute(
            "select kernel_name, counter_name, value, dispatch_id, start, end from counters_collection"):
        k = short(n)
        if k.split("<")[0] in CHAIN:
            d[k][c].append((disp, v, (e - s) / 1e3))
    out = {}
    for k, cs in d.items():
        def last(c):
            v = sorted(cs.get(c, []))[-6:]
            return (sum(x[1] for x in v) / len(v), sum(x[2] for x in v) / len(v)) if v else (None, None)
        cyc, dur = last("GRBM_GUI_ACTIVE")
        miss, _ = last("TCP_UTCL1_TRANSLATION_MISS_sum")
        hit, _ = last("TCP_UTCL1_TRANSLATION_HIT_sum")
        out[k] = (cyc, dur, miss, hit)
    return out


base = sys.argv[1]
for mode in ("pipe", "calls"):
    try:
        t = kt(base + "_%s_kt/run_results.db" % mode)
    except Exception as e:  # noqa: BLE001
        print(mode, "kt:", e)
        t = {}
    try:
        p = pmc(base + "_%s_pmc/run_results.db" % mode)
    except Exception as e:  # noqa: BLE001
        print(mode, "pmc:", e)
        p = {}
    print("== %s  (kernel us | pmc-pass us, GRBM cycles, MHz | UTCL1 miss, hit, miss rate)" % mode)
    tot = 0.0
    for k in sorted(set(t) | set(p)):
        cyc, dur, miss, hit = p.get(k, (None,) * 4)
        mhz = cyc / dur if cyc and dur else float("nan")
        rate = miss / (miss + hit) if miss is not None and hit else float("nan")
        tot += t.get(k, 0.0)
        print("%-24s %8.1f | %8.1f %10.0f %6.0f | %10.0f %10.0f %.4f" % (
            k, t.get(k, float("nan")), dur or float("nan"), cyc or float("nan"), mhz, miss or float("nan"),
            hit or float("nan"), rate))
    print("%-24s %8.1f" % ("chain", tot))
