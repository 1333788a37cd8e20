"""One-GPU proxy of the multi-GPU band partition: every rank's band of the C3 frame
(1920x1080 by default, or 3840x2160 for C4) rendered alone by a single context in band mode
(vxpt_config row_begin / row_end: the trace and denoiser over the band's rows only, no exchange),
for N = 1 / 2 / 4 / 8 bands -- the equal bands, then the cost-balanced ones bench.py runs (three rounds
of vxpt_band_balance on these same band times) -- plus the halo bytes the library's band schedule moves per rank and frame
(band_frame in vxpt_host.cpp) and their time on one xGMI link.

python tools/band_proxy.py [WIDTH HEIGHT] [--out profiles/r05_band_proxy.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
import vxpt  # noqa: E402
from bench import C1_DIR, band_tuning  # noqa: E402

XGMI_GBS = 153.0   # one xGMI link, one direction (MI355X_MICROARCH.md: 7 links x ~153 GB/s per GPU)
GROUP_US = 15.0    # latency charged per ordered RCCL group (send/recv to the neighbours), not measurable here
TRACE_ROWS, HIST_ROWS, PLANE_ROWS = 72, 2, 40   # static camera (vxpt_host.cpp band_frame)
PLANE_B = 16 + 16 + 16 + 16 + 4 + 4             # depth, normalRough, geoNormalThin, albedo, material, matParam


def atrous_rows(step):
    return step + (step // 4 if step > 4 else 0)


def halo_bytes(width, spp, rows_avail, measured=None):
    """Bytes one rank sends to ONE neighbour per frame (it receives as many), static camera, the
    library's schedule: (overlapped, in stream order).  measured: the bytes per frame vxpt_band_stats
    counted over linked contexts (ordered_groups) -- the overlapped ones are each non-last pass's tap
    records, the rest is in stream order.  Without it, the round-5 schedule's table (every chain pass
    exchanging).  rows_avail caps every depth at the bands' height (vxpt_halo_plan moves
    min(rows, both band heights))."""
    r = lambda n: min(n, rows_avail)  # noqa: E731
    # each non-last pass: its tap records beside its second half, its reservoirs after it (in order)
    overlapped = (spp - 1) * 32 * r(TRACE_ROWS) * width
    if measured is not None and rows_avail >= 72:
        return overlapped, measured - overlapped
    res_in_order = (spp - 1) * 20 * r(TRACE_ROWS)
    last = 32 * r(TRACE_ROWS) + 16 * r(2) + 20 * r(2) + PLANE_B * r(PLANE_ROWS)
    ff = 20 * r(TRACE_ROWS) + 16 * r(2)                           # filtered reservoirs + radiance
    ta = 16 * r(34) + 16 * r(2)                                   # ping for the history fix, pong
    hf = 16 * r(2)
    hc = (16 + 16 + 4) * r(HIST_ROWS)
    at = 16 * r(atrous_rows(2)) + 16 * r(atrous_rows(4)) + 16 * r(atrous_rows(8))
    ordered = (res_in_order + last + ff + ta + hf + hc + at) * width
    return overlapped, ordered


def band_rows(h, n, k):
    per = (h + 8 * n - 1) // (8 * n) * 8
    y0 = min(h, k * per)
    return y0, min(h, y0 + per)


def time_band(w, h, rows, frames, warmup, spp, tune, rccl=True):
    """One band's frames alone.  rccl: through a one-rank RCCL communicator on the band's rows --
    band_frame's schedule, the one every rank of a multi-GPU run executes (its exchange groups with
    no neighbour: the stream structure without the bytes); otherwise a plain context in band mode
    (the single-context pipelined loop, what round 4 measured)."""
    pos = tuple(p * 4 for p in (35.6184, 11.8733, 42.0387))
    r = vxpt.Renderer(w, h) if rccl else vxpt.Renderer(w, h, rows=rows)
    try:
        r.load_settings()
        if tune:
            r.set_tuning(**tune)
        r.generate_terrain((8, 8, 8), height_scale=128.0, freq_den=256.0, global_y=True)
        r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
        r.set_sky()
        if rccl:
            r.band_comm_init(vxpt.band_comm_id(), 1, 0)
            r.set_band(*rows)
        p = vxpt.DenoiseParams.defaults()
        r.render_frames(0, warmup, spp, p)
        r.sync()
        t0 = time.perf_counter()
        r.render_frames(warmup, frames, spp, p)
        r.sync()
        wall = (time.perf_counter() - t0) / frames * 1e3
        t = r.timings()
        return dict(frame_ms=round(wall, 4), trace_ms=round(t["trace_ms"], 4), denoise_ms=round(t["denoise_ms"], 4))
    finally:
        r.close()


def ordered_groups(w, h, spp, frames=3, tune=None):
    """Exchange groups per frame of the library's band schedule, counted by vxpt_band_stats over two
    linked contexts (the same band_frame code as the RCCL path): (ordered, overlapped, bytes one band
    sends its neighbour per frame)."""
    pos = tuple(p * 4 for p in (35.6184, 11.8733, 42.0387))
    rs = []
    try:
        for _ in range(2):
            r = vxpt.Renderer(w, h)
            r.load_settings()
            if tune:
                r.set_tuning(**tune)
            r.generate_terrain((8, 8, 8), height_scale=128.0, freq_den=256.0, global_y=True)
            r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
            r.set_sky()
            rs.append(r)
        linked = vxpt.LinkedBands(rs)
        p = vxpt.DenoiseParams.defaults()
        linked.render_frame(0, spp, p)  # frame 0 has its own extra exchange (the history seed)
        for r in rs:
            r.band_stats_enable(True)
        for f in range(1, 1 + frames):
            linked.render_frame(f, spp, p)
        st = rs[0].band_stats()
        # linked contexts exchange every group in stream order; on the RCCL path each non-last pass's
        # tap records go beside its second half (spp - 1 groups off the critical path) and every other
        # group -- those passes' reservoirs included -- sits between two dependent kernels
        per = st["groups"] / st["frames"]
        return per - (spp - 1), spp - 1, st["bytes_down"] / st["frames"]
    finally:
        for r in rs:
            r.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("size", nargs="*", type=int, default=[1920, 1080])
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--out", default=None)
    ap.add_argument("--tune", action="append", default=[], metavar="FIELD=VALUE")
    ap.add_argument("--plain", action="store_true",
                    help="time every band through a plain band-mode context (the single-context loop) instead of "
                         "a one-rank RCCL communicator's band_frame schedule")
    a = ap.parse_args()
    tune = {k: int(v) for k, v in (t.split("=", 1) for t in a.tune)}
    w, h = a.size
    g_ord, g_ov, sent = ordered_groups(w, h, a.spp, tune=tune)
    group_ms = g_ord * GROUP_US * 1e-3
    res = {"what": "one-GPU proxy of the band partition: each rank's band of the C3 frame rendered alone "
                   "(N > 1: through a one-rank RCCL communicator, band_frame's schedule with no neighbour; N = 1: "
                   "the single-context loop), and the halo bytes per rank and frame of the "
                   "library's schedule on one xGMI link (%.0f GB/s per direction), plus %.0f us per ordered "
                   "exchange group (RCCL group latency, charged, not measured)" % (XGMI_GBS, GROUP_US),
           "width": w, "height": h, "spp": a.spp, "tuning": tune or "defaults (bands: bench.band_tuning)",
           "groups_per_frame": {"ordered": g_ord, "overlapped": g_ov, "counted_by": "vxpt_band_stats, 2 linked contexts"},
           "bytes_per_neighbour_per_frame": round(sent), "bytes_counted_by": "vxpt_band_stats, 2 linked contexts",
           "group_latency_ms_per_frame": round(group_ms, 4),
           "ranks": {}}
    one = None

    def measure(n, bands):
        per = []
        for k, rows in enumerate(bands):
            tn = dict(tune)
            for f, v in band_tuning(w, h, n).items():  # bench.py's banded runs
                tn.setdefault(f, v)
            t = time_band(w, h, rows, a.frames, a.warmup, a.spp, tn, rccl=n > 1 and not a.plain)
            t.update(rank=k, rows=list(rows))
            per.append(t)
            print(n, k, rows, t, flush=True)
        return per

    for n in (1, 2, 4, 8):
        bands = [band_rows(h, n, k) for k in range(n)]
        per = measure(n, bands)
        balanced = None
        if n > 1:
            splits, cost, eq = [b[0] for b in bands] + [h], None, per
            for _ in range(3):
                splits, cost = vxpt.band_balance(h, splits, [t["frame_ms"] for t in per], cost)
                per = measure(n, list(zip(splits[:-1], splits[1:])))
            balanced = {"band_rows": splits, "slowest_band_ms": max(t["frame_ms"] for t in per)}
            per, balanced_per = eq, per
        slow = max(per, key=lambda t: t["frame_ms"])
        min_rows = min(y1 - y0 for y0, y1 in bands)
        ov, od = halo_bytes(w, a.spp, min_rows, sent) if n > 1 else (0, 0)
        # an interior rank talks to two neighbours over two links at once: the time of one link's bytes
        link_ms_ordered = od / (XGMI_GBS * 1e9) * 1e3
        link_ms_overlapped = ov / (XGMI_GBS * 1e9) * 1e3
        proj = slow["frame_ms"] + link_ms_ordered + (group_ms if n > 1 else 0.0)
        if n == 1:
            one = slow["frame_ms"]
        if balanced:
            balanced["bands"] = balanced_per
            balanced["projected_frame_ms"] = round(balanced["slowest_band_ms"] + link_ms_ordered + group_ms, 4)
            balanced["projected_speedup"] = round(one / balanced["projected_frame_ms"], 3)
        res["ranks"][str(n)] = {
            "balanced": balanced,
            "bands": per, "slowest_band_ms": slow["frame_ms"], "mean_band_ms": round(sum(t["frame_ms"] for t in per) / n, 4),
            "halo_mb_per_neighbour_per_frame": {"overlapped": round(ov / 1e6, 3), "in_stream_order": round(od / 1e6, 3)},
            "link_ms": {"overlapped": round(link_ms_overlapped, 4), "in_stream_order": round(link_ms_ordered, 4)},
            "projected_frame_ms": round(proj, 4),
            "projected_speedup": round(one / proj, 3) if one else None,
            "balanced_speedup_bound": round(one / (sum(t["frame_ms"] for t in per) / n + link_ms_ordered +
                                                   (group_ms if n > 1 else 0.0)), 3)
            if one else None,
        }
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
