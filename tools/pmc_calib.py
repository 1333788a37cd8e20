"""Calibration factors of rocprofv3's FETCH_SIZE / WRITE_SIZE per access width on this GPU.

Usage: python tools/pmc_calib.py FETCH_DB WRITE_DB OUT_JSON
  FETCH_DB / WRITE_DB: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE runs (separate passes) of
  tools/calib/pmc_calib (each kernel streams a known 512 MiB with one access width).
factor = known bytes / reported bytes: multiply a reported byte count by the factor of the access
width that produced it (MI355X_MICROARCH.md, HBM: 16-B-per-lane reads report half their bytes;
other widths are to be calibrated in the access pattern at hand).
"""
import json
import sqlite3
import sys

KNOWN = 512 << 20
WIDTH = {"k_read<float>": 4, "k_read<HIP_vector_type<float, 2u> >": 8, "k_read<HIP_vector_type<float, 4u> >": 16,
         "k_write<float>": 4, "k_write<HIP_vector_type<float, 4u> >": 16}


def per_kernel(path, counter):
    cur = sqlite3.connect(path).cursor()
    out = {}
    for kn, cn, v in cur.execute("select kernel_name, counter_name, value from counters_collection"):
        if cn != counter:
            continue
        name = kn.split("(")[0].replace("void ", "")
        out[name] = out.get(name, 0.0) + v * 1024.0  # FETCH_SIZE / WRITE_SIZE are in KiB
    return out


def main():
    fetch_db, write_db, out = sys.argv[1:4]
    f, w = per_kernel(fetch_db, "FETCH_SIZE"), per_kernel(write_db, "WRITE_SIZE")
    res = {"what": "known bytes / reported bytes, %d MiB streamed per kernel (tools/calib/pmc_calib.hip)" % (KNOWN >> 20),
           "fetch": {}, "write": {}}
    for name, wd in WIDTH.items():
        if name.startswith("k_read") and f.get(name):
            res["fetch"][str(wd)] = KNOWN / f[name]
        if name.startswith("k_write") and w.get(name):
            res["write"][str(wd)] = KNOWN / w[name]
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
