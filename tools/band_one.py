"""One band of the C3 frame rendered alone (band_proxy.time_band, bench.band_tuning's schedule for N
bands): python tools/band_one.py ROW0 ROW1 [N] [FIELD=VALUE ...] -- a quick A/B of a library build
(VXPT_LIB=... selects the build) or of tuning fields on a band."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from band_proxy import band_tuning, time_band  # noqa: E402


def main():
    y0, y1 = int(sys.argv[1]), int(sys.argv[2])
    rest = sys.argv[3:]
    n = int(rest.pop(0)) if rest and "=" not in rest[0] else 8
    tune = band_tuning(1920, 1080, n)
    extra = {k: int(v) for k, v in (t.split("=", 1) for t in rest)}
    tune.update(extra)
    res = [time_band(1920, 1080, (y0, y1), 12, 6, 4, tune) for _ in range(2)]
    print(json.dumps({"lib": os.path.basename(os.environ.get("VXPT_LIB", "libvxpt.so")), "rows": [y0, y1],
                      "tune": extra, "runs": res}))


if __name__ == "__main__":
    main()
