"""The denoiser chain's kernels in a rocprofv3 kernel-trace database: mean duration over the last K
launches of each (steady-state frames), and their sum.  Usage: chain_kt.py run_results.db [K]"""
import sqlite3
import sys

K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
CHAIN = ("k_firefly", "k_temporal", "k_history_fix", "k_history_clamp", "k_atrous_smem", "k_atrous_tile", "k_atrous_24",
         "k_atrous", "k_firefly_apply")
db = sqlite3.connect(sys.argv[1])
rows = list(db.execute("select name, duration from kernels order by start"))
per = {}
for n, d in rows:
    n = n.replace("vx::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    base = n.split("<")[0]
    if base in CHAIN:
        per.setdefault(n, []).append(d / 1e3)
tot = 0.0
for n, v in per.items():
    m = sum(v[-K:]) / len(v[-K:])
    tot += m
    print("%-32s %8.2f us" % (n[:32], m))
print("%-32s %8.2f us" % ("chain", tot))
