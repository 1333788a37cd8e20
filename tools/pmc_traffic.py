"""HBM traffic of the denoiser chain per frame from rocprofv3 PMC passes.

Usage: python tools/pmc_traffic.py FETCH_DB WRITE_DB STATS_DB FRAMES OUT_JSON
  FETCH_DB / WRITE_DB: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE runs (separate passes) of
  `bench.py --warmup W --steps S --no-cpu-baseline`; STATS_DB: a --kernel-trace run of the same
  command.  Only the last FRAMES frames' dispatches are used (steady state: converged history).
Correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE (KiB) is doubled -- gfx950 tallies the 128-B
requests of 16-B-per-lane loads at 64 B; WRITE_SIZE is taken as reported.
"""
import collections
import json
import sqlite3
import sys

CHAIN = ["k_world_pos", "k_firefly", "k_firefly_apply", "k_temporal", "k_history_fix", "k_history_clamp",
         "k_atrous_smem", "k_atrous"]
PER_FRAME = {"k_atrous": 3}
B_ALG = 568


def short(n):
    return n.replace("vx::(anonymous namespace)::", "").split("(")[0]


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


def main():
    fetch_db, write_db, stats_db, frames, out = sys.argv[1:6]
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
        kern[k] = {"launches_per_frame": PER_FRAME.get(k, 1), "fetch_bytes": fb, "fetch_bytes_x2": 2 * fb,
                   "write_bytes": wb, "duration_ns_per_frame": ns}
        total_f += 2 * fb
        total_w += wb
        total_ns += ns
    res = {
        "what": "HBM traffic of the denoiser chain per 1080p frame (C3), rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                "in separate passes, last %d frames (steady state)" % frames,
        "correction": "FETCH_SIZE (KiB) x 2: gfx950 tallies 128-B requests of 16-B/lane loads at 64 B "
                      "(MI355X_MICROARCH.md, HBM); WRITE_SIZE as reported",
        "kernels": kern,
        "traffic_bytes_per_frame": total_f + total_w,
        "algorithmic_bytes_per_frame": B_ALG * 1920 * 1080,
        "chain_kernel_ns_per_frame": total_ns,
    }
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print("traffic %.3f GB/frame (alg %.3f GB), chain kernels %.1f us" % (
        res["traffic_bytes_per_frame"] / 1e9, res["algorithmic_bytes_per_frame"] / 1e9, total_ns / 1e3))


if __name__ == "__main__":
    main()
