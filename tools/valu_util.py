"""Per-kernel VALU issue utilisation of the trace pass (trace_valu_util) from rocprofv3 runs.

Usage: python tools/valu_util.py SQ_DB KT_DB [OUT_JSON]
  SQ_DB: a --pmc run with SQ_INSTS_VALU (and, where the device has it, SQ_THREAD_CYCLES_VALU /
  SQ_ACTIVE_INST_VALU) of `bench.py --warmup W --steps S --no-cpu-baseline`; KT_DB: a --kernel-trace
  run of the same command (kernel durations).
issue util = SQ_INSTS_VALU x 4 cycles (a wave64 VALU op occupies a 16-lane SIMD for 4 cycles)
             / (kernel duration x 2.4 GHz x 1024 SIMDs)   -- the share of the chip's VALU issue slots used
lane util  = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU x 4)  -- active lanes per issued op
             (divergence), when both counters were collected.
"""
import collections
import json
import sqlite3
import sys

CLOCK_HZ, SIMDS = 2.4e9, 1024
TRACE = ["k_closest", "k_shade", "k_nee", "k_restir", "k_finish", "k_queue<true>", "k_queue<false>",
         "k_resume<true>", "k_resume<false>", "k_mesh_slots", "k_mesh_queue<true>", "k_mesh_queue<false>"]


def short(n):
    n = n.replace("vx::(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
    # the default (cube-table) walks: k_queue<true, false> -> k_queue<true>, k_closest<false> -> k_closest
    return n.replace(", false>", ">").replace("k_closest<false>", "k_closest")


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
            row["issue_util"] = round(c["SQ_INSTS_VALU"] * 4 / (t * CLOCK_HZ * SIMDS), 4)
        if c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU"):
            row["lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * 4 * c["SQ_ACTIVE_INST_VALU"]), 4)
        out[k] = row
    tot_t = sum(r["avg_us"] for r in out.values())
    agg = sum(r.get("issue_util", 0) * r["avg_us"] for r in out.values()) / max(tot_t, 1e-9)
    res = {"trace_valu_util": round(agg, 4), "kernels": out,
           "note": "issue util = SQ_INSTS_VALU x 4 / (duration x 2.4 GHz x 1024 SIMDs), time-weighted over the trace kernels"}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
