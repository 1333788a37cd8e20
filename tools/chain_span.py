"""Each denoiser chain's span in a rocprofv3 kernel-trace database of a pipelined bench run: from the
chain's first kernel's start (k_firefly) to its last kernel's end (the output a-trous), the sum of
its kernels' durations, and the gap in between -- to set against the bench's event-timed
denoise_ms of the same run.  Usage: chain_span.py run_results.db"""
import sqlite3
import sys

CHAIN = ("k_firefly", "k_temporal", "k_history_fix", "k_history_clamp", "k_atrous_smem", "k_atrous_tile",
         "k_atrous", "k_firefly_apply", "k_frame0", "k_copy_output")
db = sqlite3.connect(sys.argv[1])
rows = list(db.execute("select name, start, end from kernels order by start"))


def base(n):
    return n.replace("vx::(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("<")[0]


chains, cur = [], None
for n, s, e in rows:
    b = base(n)
    if b == "k_firefly":
        if cur:
            chains.append(cur)
        cur = {"start": s, "end": e, "sum": 0.0, "n": 0, "other": 0}
    if cur is None:
        continue
    if b in CHAIN:
        cur["end"] = max(cur["end"], e)
        cur["sum"] += (e - s) / 1e3
        cur["n"] += 1
    elif s < cur["end"]:
        cur["other"] += 1  # a non-chain kernel started inside the chain's span
if cur:
    chains.append(cur)
for k, c in enumerate(chains):
    span = (c["end"] - c["start"]) / 1e3
    print("chain %2d: span %7.1f us, kernels %7.1f us (%d), gaps %6.1f us, other kernels inside %d"
          % (k, span, c["sum"], c["n"], span - c["sum"], c["other"]))
if len(chains) > 2:
    steady = chains[2:]
    print("steady mean span %.1f us, kernels %.1f us" % (sum((c["end"] - c["start"]) / 1e3 for c in steady) / len(steady),
                                                        sum(c["sum"] for c in steady) / len(steady)))
