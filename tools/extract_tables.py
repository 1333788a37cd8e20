#!/usr/bin/env python3
"""Extract the numeric lookup tables the hot path needs from the reference tree
into little binary blobs under data/tables/.

These are DATA (blue-noise sample tables and spectral sky-model fit
coefficients), not source: the product loads them at run time exactly like the
reference uploads them to the GPU.

  * blue-noise sampler tables, OPTIMIZED_BLUE_NOISE_SPP == 4 section of
    renderer/util/RandGenData.h:15-39 (Heitz et al. 2019 "A low-discrepancy
    sampler that distributes Monte Carlo errors as a blue noise"):
        bn_sobol.u8      256*256      (sobol_256spp_256d)
        bn_scramble.u8   128*128*8    (scramblingTile)
        bn_rank.u8       128*128*8    (rankingTile)
  * sky model tables, renderer/sky/SkyData.h:3,556,629,2442:
        sky_datasets.f32        540   (skyDataSets)
        sky_datasets_rad.f32     60   (skyDataSetsRad)
        solar_datasets.f32     1800   (hSolarDatasets)
        limb_darkening.f32       60   (hLimbDarkeningDatasets)

Run once in the build container (the reference is absent on the GPU box);
the outputs are committed.
"""
import os
import re
import sys

import numpy as np

REF = os.environ.get("VXPT_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data", "tables")


def _array_body(text, name):
    m = re.search(r"\b%s\s*\[[^\]]*\]\s*=\s*\{(.*?)\};" % re.escape(name), text, re.S)
    if not m:
        raise RuntimeError("table %s not found" % name)
    return m.group(1)


def _ints(body):
    vals = [int(t) for t in re.findall(r"-?\d+", body)]
    return np.asarray(vals, dtype=np.int64)


def _floats(body):
    toks = re.findall(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?", body)
    # C float literal semantics: decimal -> nearest binary32
    return np.asarray([float(t) for t in toks], dtype=np.float64).astype(np.float32)


def main():
    os.makedirs(OUT, exist_ok=True)
    rg = open(os.path.join(REF, "renderer/util/RandGenData.h")).read()
    start = rg.index("#if OPTIMIZED_BLUE_NOISE_SPP == 4")
    sec = rg[start:]
    for name, fname, n in (("h_sobol_256spp_256d", "bn_sobol.u8", 256 * 256),
                           ("h_scramblingTile", "bn_scramble.u8", 128 * 128 * 8),
                           ("h_rankingTile", "bn_rank.u8", 128 * 128 * 8)):
        v = _ints(_array_body(sec, name))
        assert v.size == n, (name, v.size)
        assert v.min() >= 0 and v.max() <= 255
        v.astype(np.uint8).tofile(os.path.join(OUT, fname))

    sky = open(os.path.join(REF, "renderer/sky/SkyData.h")).read()
    for name, fname, n in (("skyDataSets", "sky_datasets.f32", 540),
                           ("skyDataSetsRad", "sky_datasets_rad.f32", 60),
                           ("hSolarDatasets", "solar_datasets.f32", 1800),
                           ("hLimbDarkeningDatasets", "limb_darkening.f32", 60)):
        v = _floats(_array_body(sky, name))
        assert v.size == n, (name, v.size)
        v.astype("<f4").tofile(os.path.join(OUT, fname))
    print("tables written to", os.path.abspath(OUT))
    return 0


if __name__ == "__main__":
    sys.exit(main())
