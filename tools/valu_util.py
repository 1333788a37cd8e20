"""Per-kernel VALU issue utilisation of the trace pass (trace_valu_util) from rocprofv3 runs.

Usage: python tools/valu_util.py SQ_DB KT_DB [OUT_JSON]
  SQ_DB: a --pmc run with SQ_INSTS_VALU (and, where the device has it, SQ_THREAD_CYCLES_VALU /
  SQ_ACTIVE_INST_VALU) of `bench.py --warmup W --steps S --no-cpu-baseline`; KT_DB: a --kernel-trace
  run of the same command (kernel durations).
issue util = SQ_INSTS_VALU x 2 cycles (gfx950: a wave64 VALU op issues over 2 cycles on a SIMD-32;
             MI355X_MICROARCH.md constants table) / (kernel duration x 2.4 GHz x 1024 SIMDs)
             -- the share of the chip's VALU issue slots used
lane util  = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)  -- active lanes per issued op
             (divergence), when both counters were collected (both count in the same unit).
"""
import collections
import json
import re
import sqlite3
import sys

CLOCK_HZ, SIMDS = 2.4e9, 1024
TRACE = ["k_closest", "k_shade", "k_nee", "k_restir", "k_finish", "k_queue<true>", "k_queue<false>",
         "k_resume<true>", "k_resume<false>", "k_mesh_slots", "k_mesh_queue<true>", "k_mesh_queue<false>"]


def short(n):
    """Kernel name without namespace and walk-table template argument: k_queue<true, true> and
    k_queue<true, false> -> k_queue<true>, k_closest<true> -> k_closest, k_shade<false> -> k_shade
    (k_shade<true>, the instanced-mesh variant -> k_shade<mesh>)."""
    n = n.replace("vx::(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
    m = re.match(r"(k_queue|k_resume)<(true|false), (true|false)>", n)
    if m:
        return "%s<%s>" % (m.group(1), m.group(2))
    m = re.match(r"(k_closest|k_shade|k_nee|k_restir)<(true|false)>", n)
    if m:
        return m.group(1) if (m.group(1) == "k_closest" or m.group(2) == "false") else m.group(1) + "<mesh>"
    return n


def main():
    sq_db, kt_db = sys.argv[1:3]
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for kn, cn, v in sqlite3.connect(sq_db).cursor().execute(
            "select kernel_name, counter_name, value from counters_collection"):
        cnt[short(kn)][cn].append(v)
    dur = collections.defaultdict(list)
    for n, d in sqlite3.connect(kt_db).cursor().execute("select name, duration from kernels"):
        dur[short(n)].append(d)
    out = {}
    for k in TRACE:
        if k not in cnt or k not in dur:
            continue
        c = {n: sum(v) / len(v) for n, v in cnt[k].items()}
        t = sum(dur[k]) / len(dur[k]) * 1e-9
        row = {"avg_us": round(t * 1e6, 2), "valu_insts": c.get("SQ_INSTS_VALU")}
        if c.get("SQ_INSTS_VALU"):
            row["issue_util"] = round(c["SQ_INSTS_VALU"] * 2 / (t * CLOCK_HZ * SIMDS), 4)
        if c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU"):
            row["lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 4)
        out[k] = row
    # chip level: the trace kernels' VALU instructions over the time any of them runs (the union of
    # their dispatch intervals: with two streams a pass's halves overlap, so per-kernel durations
    # double-count the wall time)
    ivs = sorted((s0, e0) for n, s0, e0 in sqlite3.connect(kt_db).cursor().execute(
        "select name, start, end from kernels") if short(n) in TRACE for _ in [0])
    busy, cs, ce = 0, None, None
    for s0, e0 in ivs:
        if cs is None or s0 > ce:
            busy += (ce - cs) if cs is not None else 0
            cs, ce = s0, e0
        else:
            ce = max(ce, e0)
    busy += (ce - cs) if cs is not None else 0
    ndisp = collections.Counter(short(n) for (n,) in sqlite3.connect(kt_db).cursor().execute("select name from kernels"))
    insts = sum(r["valu_insts"] * ndisp[k] for k, r in out.items() if r.get("valu_insts"))
    chip = insts * 2 / (busy * 1e-9 * CLOCK_HZ * SIMDS) if busy else None
    tot_t = sum(r["avg_us"] for r in out.values())
    lanes = [r for r in out.values() if "lane_util" in r]
    lane_agg = (sum(r["lane_util"] * r["avg_us"] for r in lanes) / sum(r["avg_us"] for r in lanes)) if lanes else None
    agg = sum(r.get("issue_util", 0) * r["avg_us"] for r in out.values()) / max(tot_t, 1e-9)
    res = {"trace_valu_util": round(chip, 4) if chip else round(agg, 4),
           "trace_valu_lane_util": round(lane_agg, 4) if lane_agg else None,
           "kernel_time_weighted_issue_util": round(agg, 4),
           "kernels": out,
           "note": "trace_valu_util = the trace kernels' SQ_INSTS_VALU x 2 cycles / (the time any trace kernel runs x 2.4 GHz x 1024 SIMDs); per kernel issue util = SQ_INSTS_VALU x 2 / (its duration x 2.4 GHz x 1024) -- with the pass halves on two streams a kernel's duration includes the other stream's work; lane util = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU), time-weighted"}
    if len(sys.argv) > 4:  # the profiled bench run's log: its mode (bench.py attaches matching modes only)
        from pmc_traffic import bench_mode
        res["mode"] = bench_mode(sys.argv[4])
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
