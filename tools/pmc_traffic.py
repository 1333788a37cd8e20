"""HBM traffic of the denoiser chain per frame from rocprofv3 PMC passes.

Usage: python tools/pmc_traffic.py FETCH_DB WRITE_DB STATS_DB FRAMES OUT_JSON [CALIB_JSON [BENCH_LOG]]
  BENCH_LOG: the profiled bench run's output; its line's `mode` is recorded, and bench.py attaches
  the result only to lines of the same mode.
  FETCH_DB / WRITE_DB: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE runs (separate passes) of
  `bench.py --warmup W --steps S --no-cpu-baseline`; STATS_DB: a --kernel-trace run of the same
  command.  Only the last FRAMES frames' dispatches are used (steady state: converged history).
Correction (MI355X_MICROARCH.md, HBM): the reported bytes depend on the access width (16-B-per-lane
reads report half).  CALIB_JSON (tools/pmc_calib.py) holds the measured factor per width; each
kernel's FETCH_SIZE is corrected with its own mix of load widths (LOAD_MIX: the share of its
algorithmic read bytes loaded 4 / 16 bytes per lane): reported = sum_w actual_w / factor_w with
actual_w = A * share_w, so A = reported / sum_w (share_w / factor_w).  Without a calibration file
FETCH_SIZE is doubled (the guide's 16-B figure) and marked as an upper bound.
"""
import collections
import json
import sqlite3
import sys

CHAIN = ["k_firefly", "k_firefly_filter", "k_firefly_apply", "k_temporal", "k_history_fix", "k_history_clamp",
         "k_atrous_smem", "k_atrous_tile<2, 16>", "k_atrous_tile<4, 16>", "k_atrous"]
PER_FRAME = {}
B_ALG = 568
# share of each kernel's algorithmic read bytes by load width (bytes per lane), from its loads:
# firefly: depth 4 + 16-bit material + reservoir (16 + 4) ; temporal: depth, 12 previous depths and 4
# history lengths (4 B) beside 16-B planes; the stencils: depth + history length (4 B) beside
# 16-B planes (ASmem: + the 4-B material plane)
LOAD_MIX = {"k_firefly": {4: 10 / 26, 16: 16 / 26}, "k_temporal": {4: 12 / 124, 16: 112 / 124},
            "k_history_fix": {4: 0.2, 16: 0.8}, "k_history_clamp": {4: 8 / 56, 16: 48 / 56},
            "k_atrous_smem": {4: 12 / 60, 16: 48 / 60}, "k_atrous_tile<2, 16>": {4: 8 / 56, 16: 48 / 56},
            "k_atrous_tile<4, 16>": {4: 8 / 56, 16: 48 / 56}, "k_atrous": {4: 8 / 56, 16: 48 / 56}}


def short(n):
    n = n.replace("vx::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    # the tile-size / tile-order template arguments of the LDS stencils are not part of the pass
    for base in ("k_history_clamp", "k_atrous_smem", "k_temporal", "k_firefly"):
        if n.startswith(base + "<"):
            return base
    return n


def counters(path, name):
    cur = sqlite3.connect(path).cursor()
    vals = collections.defaultdict(list)
    for kn, cn, v, disp in cur.execute(
            "select kernel_name, counter_name, value, dispatch_id from counters_collection order by dispatch_id"):
        if cn == name:
            vals[short(kn)].append(v)
    return vals


def durations(path):
    cur = sqlite3.connect(path).cursor()
    d = collections.defaultdict(list)
    for n, dur in cur.execute("select name, duration from kernels order by start"):
        d[short(n)].append(dur)
    return d


def bench_mode(log):
    """The `mode` of the last bench.py JSON line in a log."""
    lines = [ln for ln in open(log) if ln.startswith("{")]
    return json.loads(lines[-1]).get("mode") if lines else None


def main():
    fetch_db, write_db, stats_db, frames, out = sys.argv[1:6]
    calib, mode = None, None
    if len(sys.argv) > 6:
        with open(sys.argv[6]) as fc:
            calib = json.load(fc)
    if len(sys.argv) > 7:
        mode = bench_mode(sys.argv[7])
    frames = int(frames)
    fetch, write, dur = counters(fetch_db, "FETCH_SIZE"), counters(write_db, "WRITE_SIZE"), durations(stats_db)
    kern, total_f, total_w, total_ns = {}, 0.0, 0.0, 0.0
    for k in CHAIN:
        n = PER_FRAME.get(k, 1) * frames
        f = fetch.get(k, [])[-n:]
        w = write.get(k, [])[-n:]
        t = dur.get(k, [])[-n:]
        if not f:
            continue
        fb = sum(f) * 1024.0 / frames
        wb = sum(w) * 1024.0 / frames
        ns = sum(t) / frames
        if calib:
            mix = LOAD_MIX.get(k, {16: 1.0})
            fc = fb / sum(sh / calib["fetch"][str(wd)] for wd, sh in mix.items())
            wc = wb * calib["write"]["16"]
        else:
            fc, wc = 2 * fb, wb
        kern[k] = {"launches_per_frame": PER_FRAME.get(k, 1), "fetch_bytes_reported": fb, "fetch_bytes": fc,
                   "write_bytes_reported": wb, "write_bytes": wc, "duration_ns_per_frame": ns}
        total_f += fc
        total_w += wc
        total_ns += ns
    res = {
        "what": "HBM traffic of the denoiser chain per 1080p frame (C3), rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                "in separate passes, last %d frames (steady state)" % frames,
        "correction": ("per-kernel FETCH_SIZE corrected with the calibrated factor of each load width weighted by "
                       "the kernel's load mix; WRITE_SIZE x the 16-B store factor; calibration: %s" % json.dumps(calib))
                      if calib else "FETCH_SIZE x 2 (upper bound: the 16-B/lane figure applied to every load); "
                                    "WRITE_SIZE as reported",
        "kernels": kern,
        "traffic_bytes_per_frame": total_f + total_w,
        "algorithmic_bytes_per_frame": B_ALG * 1920 * 1080,
        "chain_kernel_ns_per_frame": total_ns,
        "mode": mode,
    }
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print("traffic %.3f GB/frame (alg %.3f GB), chain kernels %.1f us" % (
        res["traffic_bytes_per_frame"] / 1e9, res["algorithmic_bytes_per_frame"] / 1e9, total_ns / 1e3))


if __name__ == "__main__":
    main()
