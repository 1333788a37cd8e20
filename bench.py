"""Benchmark of the offline hot path (BASELINE.json metric).

Workload (default = BASELINE config C3): 1920x1080, 4 spp full path (voxel DDA +
Disney BSDF + NEE/ReSTIR-DI, bounce limits 3/1 as RayGen.cu:146-147) + ReLAX
denoiser (TA, history fix, clamping, a-trous 1+3), synthetic 256^3 Perlin voxel
world (8x8x8 chunks, C1 terrain scaled x4: heights 128, freq 1/256, world-y
heights), camera = C1 camera with position x4.  One step = one
OfflineBackend::renderFrame = 4 trace passes + 1 denoise.

value = whole-job Mpaths/s = W*H*spp * K / max-over-ranks wall time of K steps.
roofline = the denoiser chain (HBM-bound): algorithmic bytes 568 B/px * W*H per
frame / its HIP-event duration on the context's stream.
cpu_baseline = the oracle (C++ restatement, OpenMP) tracing a bounded band of
rows of the same frame on this host's cores (rank 0, N=1 only).

Multi-GPU (N>1, launched by torch.distributed.run): the frame is split into N
horizontal bands; each rank's library context renders its band and enqueues
the halo exchanges itself (RCCL over xGMI: grouped send/recv with the band
neighbours on the context stream, vxpt_band_comm_init).  Total work is fixed
(strong scaling); value = whole-frame paths / max-over-ranks time; roofline =
the rank's band (its denoiser time includes the exchanges).  Before the run the
band boundaries are balanced (vxpt_band_balance): every rank times its band of
the frame alone (no exchange), the ranks share the times, and the boundaries
move to equalise them -- rows near the horizon cost several times the ground's,
so equal bands leave the slowest rank far above the mean (--equal-bands: off).
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))

B_ALG_PER_PX = 568  # D1 24 + D2 4 + D3 148 + D4 8 + D5 92 + D6 60 + D7 180 + D8 52
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
C1_POS = (35.6184, 11.8733, 42.0387)
C1_DIR = (-0.321564, -0.0129988, -0.946799)


def scene_args(a):
    """(chunks, height scale, frequency denominator, world-y heights, camera position) of the run's
    scene: c1 = mainOffline's default scene (2x1x2 chunks, VoxelSceneGen.cu:341-388's terrain; SURVEY
    §8d C1 / C2 / C5), c3 = the 256^3 world (C1 terrain scaled by world/64: heights and frequency
    scaled, world-y heights, camera position scaled)."""
    if a.scene == "c1":
        return (2, 1, 2), 32.0, 64.0, False, C1_POS
    scale = a.world // 64
    pos = tuple(p * scale for p in C1_POS)
    chunks = (a.world // 32, a.world // 32, a.world // 32)
    return chunks, 32.0 * scale, 64.0 * scale, True, pos


def run_mode(a, spp):
    """What a committed profile must have been measured on to be attached to this run's line."""
    return {"scene": a.scene, "world": a.world if a.scene == "c3" else 64, "width": a.width, "height": a.height,
            "spp": spp, "bounces": "%d/%d" % a.bounce_limits, "primary_only": bool(a.primary_only),
            "tune": dict(sorted(a.tune.items()))}


def matching_profile(pattern, mode):
    """The newest committed profile JSON under profiles/ whose recorded `mode` equals this run's
    (tools/pmc_traffic.py / valu_util.py copy it from the profiled bench line), or (None, None)."""
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", pattern)), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("mode") == mode:
            return d, os.path.relpath(path, REPO)
    return None, None


def trace_roofline_profile(mode):
    """The trace's roofline (tools/trace_roofline.py -> profiles/*_trace_roofline.json) measured on this
    run's workload: its mode equals the run's but for the kernels-one-at-a-time schedule it is measured
    with (tune overlap = 0, a schedule knob that changes no result) and its frame count."""
    want = dict(mode, tune={k: v for k, v in mode["tune"].items() if k != "overlap"})
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_trace_roofline.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        m = dict(d.get("mode", {}))
        m.pop("frames", None)
        m["tune"] = {k: v for k, v in m.get("tune", {}).items() if k != "overlap"}
        if m == want:
            keep = ("bound", "unit", "achieved", "peak", "frac", "lane_util", "peak_converged", "frac_converged",
                    "steps_per_frame", "insts_per_step", "traversal_ms_per_frame", "per_path")
            out = {k: d[k] for k in keep if k in d}
            out["source"] = os.path.relpath(path, REPO)
            out["what"] = ("the traversal kernels (k_closest, k_queue, k_resume, k_resume_split), kernels one at a "
                           "time: lane DDA steps per s against the VALU-issue-bound peak (DESIGN.md §6)")
            return out
    return None


def native_oracle():
    """Build the oracle for this host with -march=native (the CPU baseline's
    flags) into oracle/_native/ -- the prebuilt liboracle.so targets x86-64-v3 because it is
    compiled in another container.  Returns (library path, march label)."""
    src = os.path.join(REPO, "oracle")
    out_dir = os.path.join(src, "_native")
    lib = os.path.join(out_dir, "liboracle_native.so")
    try:
        os.makedirs(out_dir, exist_ok=True)
        srcs = [os.path.join(src, f) for f in ("orc_scene.cpp", "orc_sky.cpp", "orc_trace.cpp", "orc_denoise.cpp",
                                               "orc_post.cpp", "orc_lights.cpp", "orc_mesh.cpp", "orc_api.cpp")]
        subprocess.run(["g++", "-O3", "-march=native", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
                        "-std=c++17", "-shared", "-o", lib] + srcs, check=True, timeout=120,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        return lib, "native"
    except (OSError, subprocess.SubprocessError):
        return os.path.join(src, "liboracle.so"), "x86-64-v3"


def cpu_baseline(a, target_s):
    lib, march = native_oracle()
    os.environ["ORACLE_LIB"] = lib
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    chunks, hs, fd, gy, pos = scene_args(a)
    o = oracle.Oracle(a.width, a.height, bounces=a.bounce_limits)
    o.terrain(chunks, height_scale=hs, freq_den=fd, global_y=gy)
    o.set_camera(pos, C1_DIR, 90.0)
    o.set_camera(pos, C1_DIR, 90.0, which=1)
    o.set_sky()
    # grow a band around the middle of the frame until it takes about target_s;
    # past a full frame, trace further 1-spp passes (iterationIndex 1, 2, ...)
    mid, rows, dt, passes = a.height // 2, 8, 0.0, 1
    while True:
        y0 = max(0, mid - rows // 2)
        t0 = time.perf_counter()
        for it in range(passes):
            o.trace(it, y0, y0 + rows, primary_only=a.primary_only)
        dt = time.perf_counter() - t0
        if dt >= 0.5 * target_s:
            break
        grow = max(2.0, target_s / max(dt, 1e-3))
        if rows < a.height:
            rows = int(min(a.height, rows * grow))
        else:
            passes = int(passes * grow) + 1
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    res = {"value": passes * rows * a.width / dt / 1e6, "unit": "Mpaths/s", "cores": cores, "kind": "port",
           "march": march,
           "sample": "oracle trace of rows [%d,%d) x %d pass(es) at %dx%d, 1 spp each, %s, same scene (%.1f s)" % (
               y0, y0 + rows, passes, a.width, a.height, "primary rays only" if a.primary_only else "full path", dt)}
    if not a.primary_only:
        # the denoiser chain on the CPU: whole-frame trace passes feed two
        # frames; the second (steady state: temporal accumulation, history fix and clamping,
        # a-trous 1 + 3 on the ReLAX defaults) is timed
        o.set_denoise_params([30, 6, 2, 0.5, 0.15, 0.003, 0.01, 0.05, 500000], [1, 1, 1, 1, 1, 1])
        o.trace(0)
        o.post_trace()
        o.denoise(0, 1)
        o.set_camera(pos, C1_DIR, 90.0, which=1)
        o.trace(1)
        o.post_trace()
        t0 = time.perf_counter()
        o.denoise(1, 2)
        res["denoise_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        res["denoise_sample"] = "oracle ReLAX chain, one steady-state %dx%d frame (frame 1)" % (a.width, a.height)
    return res


FRAME_LIMIT_S = 10.0  # watchdog: a frame (any rank) that takes longer ends the run (one takes ~6 ms)
SETUP_LIMIT_S = 300.0  # watchdog: context creation, world generation, rendezvous, the balancing renders


class Watchdog:
    """Host watchdog over the run's GPU syncs and collectives (no re-exec, no retry): a section armed
    with a limit that has not been disarmed when the limit expires prints what it was doing and ends
    the process with status 5 -- a hung halo exchange or kernel on one rank ends the driver's
    multi-GPU bench with a message instead of a hang."""

    def __init__(self, rank=0):
        self.rank, self._t = rank, None

    def arm(self, seconds, what):
        self.disarm()
        self._t = threading.Timer(seconds, self._fire, (seconds, what))
        self._t.daemon = True
        self._t.start()

    def frames(self, n, what):
        self.arm(FRAME_LIMIT_S * n + 30.0, "%s (%d frames, %.0f s per frame)" % (what, n, FRAME_LIMIT_S))

    def disarm(self):
        if self._t is not None:
            self._t.cancel()
            self._t = None

    def _fire(self, seconds, what):
        print("bench watchdog: rank %d: %s did not finish within %.0f s; exiting" % (self.rank, what, seconds),
              file=sys.stderr, flush=True)
        os._exit(5)


def band_parity(out, ref):
    """The banded run's frame gathered at the root against the single-context render of the same frame
    sequence: bit-exact per pixel (every channel's bits).  Returns the JSON fields of the check."""
    import numpy as np
    a = np.ascontiguousarray(out).view(np.uint32).reshape(out.shape[0], out.shape[1], -1)
    b = np.ascontiguousarray(ref).view(np.uint32).reshape(ref.shape[0], ref.shape[1], -1)
    if a.shape != b.shape:
        return {"band_parity": False, "mismatched_px": None, "why": "shapes %s vs %s" % (a.shape, b.shape)}
    bad = (a != b).any(axis=-1)
    res = {"band_parity": not bool(bad.any()), "mismatched_px": int(bad.sum())}
    if bad.any():
        rows = np.nonzero(bad.any(axis=1))[0]
        res["mismatched_rows"] = [int(rows[0]), int(rows[-1])]
    return res


def single_context_frames(make, frames, spp, params, primary_only=False):
    """The frame sequence a banded context rendered (frames 0 .. frames-1), in one whole-frame context:
    the reference image of band_parity.  Returns the context (the caller reads and closes it)."""
    s = make()
    if primary_only:
        s.trace(frames - 1, primary_only=True)  # primary rays: no state carried between frames
    else:
        s.render_frames(0, frames, spp, params)
    s.sync()
    return s


def band_tuning(width, height, world):
    """Schedule defaults of a rank's band (N>1).  A band is latency bound: a third wavefront state
    set lets its passes' first halves run further ahead, and below ~0.7 Mpx a third front stream
    adds overlap (1080p, 8 balanced bands: slowest band 1.52 -> 1.43 ms per frame), while bigger bands
    lose by it (1080p, 2 bands of 1 Mpx: 3.16 -> 3.22 ms; profiles/r04_band_proxy*.json); below
    ~0.4 Mpx the longest straggler walks are split across lanes (k_resume_split)."""
    if world <= 1:
        return {}
    # chain_gate 0: a frame's later first halves start as soon as their state set is free instead of
    # after the previous frame's denoiser chain -- on a band the second pass's first half was on the
    # critical path (one 8-band 1080p band 1.255 -> 1.174 ms, another 1.094 -> 0.986)
    # (resume_wg_per_cu 16: the bands' measured straggler grid; the single-GPU default is 24)
    t = {"state_sets": 3, "chain_gate": 0, "resume_wg_per_cu": 16}
    if width * height / world < 700e3:
        t["front_streams"] = 3
    if width * height / world < 400e3:
        # the round-5 walk ladder: the second straggler level after 5 + 8 iterations, its walks in 16
        # pieces (a small band's passes wait on their longest walks: 136-row 1080p band 1.40-1.42 ->
        # 1.31-1.34 ms per frame; 272 rows even: DESIGN.md §4), no third level (the library's 4 / 6 / 12
        # ladder adds a launch to each traversal's chain: 8-band 1080p bands 8-10 % slower; 2- and 4-band
        # bands gain 2-5 % with it)
        t.update(iter_cap=5, iter_cap2=8, iter_cap3=0, resume_split=16)
    return t


def balance_bands(a, make, params, world, rank, dist, rounds=3, frames=6):
    """Cost-balanced band boundaries (vxpt_band_balance): each round, every rank renders its band
    of the current partition alone in a throwaway context (band mode, no exchange: its compute
    only), the ranks all-gather the per-frame times, and every rank computes the same next
    partition from them.  Returns (row boundaries, per-round log)."""
    import vxpt
    splits, cost, log = vxpt.equal_splits(a.height, world), None, []
    for _ in range(rounds):
        r = make()
        try:
            r.set_band(splits[rank], splits[rank + 1])

            def run(f0, n):
                if a.primary_only:
                    for f in range(f0, f0 + n):
                        r.trace(f, primary_only=True)
                else:
                    r.render_frames(f0, n, a.spp, params)
                r.sync()
            run(0, 3)
            t0 = time.perf_counter()
            run(3, frames)
            ms = (time.perf_counter() - t0) / frames * 1e3
        finally:
            r.close()
        times = [None] * world
        dist.all_gather_object(times, ms)
        log.append({"band_rows": splits, "band_ms": [round(t, 4) for t in times]})
        splits, cost = vxpt.band_balance(a.height, splits, times, cost)
    log.append({"band_rows": splits})
    return splits, log


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--world", type=int, default=256, help="c3 scene: world edge in voxels (multiple of 64)")
    ap.add_argument("--primary-only", action="store_true", help="C2: primary rays + sky + G-buffer, no denoiser")
    ap.add_argument("--scene", choices=("c1", "c3"), default=None,
                    help="c1: mainOffline's default 64x32x64 scene (SURVEY §8d C2's); c3: the --world^3 world "
                         "(default: c1 with --primary-only, else c3)")
    ap.add_argument("--tune", action="append", default=[], metavar="FIELD=VALUE",
                    help="a vxpt_tuning field for this run (schedule only; results are unchanged)")
    ap.add_argument("--bounces", default="3/1",
                    help="total/diffuse bounce limits: 3/1 = the reference's (RayGen.cu:146-147); 4/4 = the "
                         "'4 bounces' of BASELINE.json's config line, labelled as such")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--equal-bands", action="store_true",
                    help="N>1: keep the equal row bands instead of balancing the boundaries on measured band times")
    ap.add_argument("--frame-calls", action="store_true",
                    help="time K vxpt_render_frame calls instead of one pipelined vxpt_render_frames(K)")
    ap.add_argument("--bands", action="store_true",
                    help="N=1: run the banded path through a one-rank RCCL communicator (the N>1 schedule, "
                         "its instrumentation and its band_parity check, with no neighbour)")
    ap.add_argument("--no-band-parity", action="store_true",
                    help="banded runs: skip the check of the gathered frame against a single-context render")
    a = ap.parse_args()
    a.bounce_limits = tuple(int(v) for v in a.bounces.split("/"))
    if a.scene is None:
        a.scene = "c1" if a.primary_only else "c3"
    a.tune = {k: int(v) for k, v in (t.split("=", 1) for t in a.tune)}
    for k, v in band_tuning(a.width, a.height, int(os.environ.get("WORLD_SIZE", 1))).items():
        a.tune.setdefault(k, v)
    assert len(a.bounce_limits) == 2 and a.bounce_limits[0] >= a.bounce_limits[1] >= 1, a.bounces

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    banded = world > 1 or a.bands
    wd = Watchdog(rank)
    wd.arm(SETUP_LIMIT_S, "setup (rendezvous, contexts, world, band balancing)")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import torch
    import vxpt
    import bands

    chunks, hs, fd, gy, pos = scene_args(a)
    params = vxpt.DenoiseParams.defaults()

    def make():
        r = vxpt.Renderer(a.width, a.height, device=local, bounces=a.bounce_limits)
        r.load_settings()
        if a.tune:
            r.set_tuning(**a.tune)
        r.generate_terrain(chunks, height_scale=hs, freq_den=fd, global_y=gy)
        r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
        r.set_sky()
        return r

    splits, balance_log = None, None
    if world > 1 and not a.equal_bands:
        splits, balance_log = balance_bands(a, make, params, world, rank, dist)
    r = make()
    band = None
    if banded:
        # the library renders this rank's band and enqueues the halo exchanges itself
        # (RCCL over xGMI on the context stream); the host only hands out the unique id
        obj = [vxpt.band_comm_id() if rank == 0 else None]
        if dist is not None:
            dist.broadcast_object_list(obj, src=0)
        err = ""
        try:
            r.band_comm_init(obj[0], world, rank, splits)
        except vxpt.VxptError as e:
            err = str(e)
        errs = [err]
        if dist is not None:
            errs = [None] * world
            dist.all_gather_object(errs, err)
        if any(errs):
            # no band communicator on some rank: no banded frame can be rendered, and N independent
            # whole frames would not be the banded workload -- fail instead of reporting them
            bad = next(e for e in errs if e)
            print("band exchange unavailable (vxpt_band_comm_init): %s" % bad, file=sys.stderr, flush=True)
            r.close()
            if dist is not None:
                dist.destroy_process_group()
            sys.exit(3)
        band = bands.band_rows(a.height, world, rank) if splits is None else (splits[rank], splits[rank + 1])
    wd.disarm()

    def step(frame):
        if a.primary_only:
            r.trace(frame, primary_only=True)
            r.sync()
        else:
            r.render_frame(frame, a.spp, params)

    frame = 0
    wd.frames(a.warmup, "warmup")
    for _ in range(a.warmup):
        step(frame)
        frame += 1
    wd.disarm()

    def barrier():
        torch.cuda.synchronize(local)
        if dist is not None:
            dist.barrier()
        r.sync()

    trace_ms, denoise_ms = [], []
    pipelined = not a.primary_only and not a.frame_calls
    wd.frames(a.steps + 2, "timed region")
    barrier()
    t0 = time.perf_counter()
    if pipelined:
        # the K frames as one vxpt_render_frames call: same work and buffers as K render_frame
        # calls, each frame's first trace pass overlapping the previous frame's last
        r.render_frames(frame, a.steps, a.spp, params)
        frame += a.steps
        t = r.timings()
        trace_ms.append(t["trace_ms"])
        denoise_ms.append(t["denoise_ms"])
    else:
        for _ in range(a.steps):
            step(frame)
            frame += 1
            t = r.timings()
            trace_ms.append(t["trace_ms"])
            denoise_ms.append(t["denoise_ms"])
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    wd.disarm()

    # bands: after the timed region, 4 more frames with the library's band instrumentation on
    # (vxpt_band_stats: every frame's trace / denoiser spans, the halo groups' HIP-event time, count and
    # bytes per neighbour) -- what the first multi-GPU run needs to explain its own scaling
    band_diag, timing_src = None, "vxpt_timings (the pipelined run's chains)" if pipelined else "vxpt_timings per frame"
    if banded and not a.primary_only:
        wd.frames(4, "band instrumentation frames")
        r.band_stats_enable(True)
        r.render_frames(frame, 4, a.spp, params)
        frame += 4
        st = r.band_stats()
        r.band_stats_enable(False)
        wd.disarm()
        nf = max(st["frames"], 1)
        mine = {"rank": rank, "rows": [st["row_begin"], st["row_end"]], "frames": st["frames"],
                "trace_ms": round(st["trace_ms"] / nf, 4), "denoise_ms": round(st["denoise_ms"] / nf, 4),
                "halo_ordered_ms": round(st["exchange_ms"] / nf, 4),
                "halo_overlapped_ms": round(st["exchange_overlap_ms"] / nf, 4),
                "halo_groups": round(st["groups"] / nf, 2), "halo_groups_ordered": round(st["groups_ordered"] / nf, 2),
                "halo_mb_up": round(st["bytes_up"] / nf / 1e6, 3), "halo_mb_down": round(st["bytes_down"] / nf / 1e6, 3)}
        ranks = [mine]
        if dist is not None:
            ranks = [None] * world
            dist.all_gather_object(ranks, mine)
        band_diag = {"frames": nf, "what": "per rank and frame, 4 banded frames after the timed region with "
                     "vxpt_band_stats on: trace / denoiser spans (with their exchanges), HIP-event time inside the "
                     "ordered and the overlapped halo groups, groups per frame, MB sent up / down",
                     "ranks": ranks}
        # every frame's spans (vxpt_timings of a banded run holds its last frame's)
        trace_ms, denoise_ms = [mine["trace_ms"]], [mine["denoise_ms"]]
        timing_src = "vxpt_band_stats over the 4 diagnostic frames (every frame's spans)"

    # banded runs check themselves: every band's rows of the last frame gathered at rank 0 (RCCL,
    # vxpt_band_gather) against one whole-frame context rendering the same frame sequence on rank 0
    # (tools/rccl_bands_check.py's check, on the benchmarked workload); a mismatch fails the run
    parity = None
    if banded and not a.no_band_parity:
        name = "DEPTH" if a.primary_only else "OUTPUT"
        wd.frames(frame + 2, "band parity (gather + single-context render of %d frames)" % frame)
        r.band_gather(name, 0)
        if rank == 0:
            s = single_context_frames(make, frame, a.spp, params, a.primary_only)
            try:
                parity = band_parity(r.read(name), s.read(name))
            finally:
                s.close()
            parity.update({"buffer": name, "frames": frame,
                           "what": "rank 0: the banded run's last frame gathered from every band (vxpt_band_gather) "
                                   "vs one whole-frame context rendering the same %d frames, bit for bit" % frame})
        if dist is not None:
            obj = [parity]
            dist.broadcast_object_list(obj, src=0)
            parity = obj[0]
        wd.disarm()
        if not parity["band_parity"]:
            print("band parity FAILED: %s" % json.dumps(parity), file=sys.stderr, flush=True)

    band_px = a.width * a.height
    if band is not None:
        band_px = a.width * (band[1] - band[0])
    spp = 1 if a.primary_only else a.spp
    paths = a.width * a.height * spp
    # single GPU / bands: the whole frame's paths per step
    value = paths * a.steps / elapsed / 1e6
    avg_trace = sum(trace_ms) / len(trace_ms)
    avg_dn = sum(denoise_ms) / len(denoise_ms)
    if a.primary_only:
        # trace-only mode: compulsory G-buffer writes (illum 16 + depth 4 + normRough 16 + geoNormal 16 +
        # matParam 16 + albedo 16 + material 4 + motion 16 = 104 B/px)
        alg_bytes, dur_ms, kern = 104 * a.width * a.height, avg_trace, "k_trace (primary only)"
    else:
        alg_bytes, dur_ms, kern = B_ALG_PER_PX * band_px, avg_dn, "denoiser chain"
    achieved = alg_bytes / (dur_ms * 1e-3) / 1e9
    # measured HBM bytes of the chain per frame: committed rocprofv3 PMC passes (tools/gpu_pmc.sh ->
    # profiles/*_pmc_denoise.json) of this same mode only; PMC cannot run inside this timed process
    mode = run_mode(a, 1 if a.primary_only else a.spp)
    traffic, traffic_src, valu, valu_src, trace_roof = None, None, None, None, None
    if not a.primary_only and not banded:
        trace_roof = trace_roofline_profile(mode)
        d, traffic_src = matching_profile("*_pmc_denoise.json", mode)
        traffic = d["traffic_bytes_per_frame"] if d else None
        # VALU issue utilisation of the trace kernels (tools/valu_util.py -> profiles/*_valu_util.json)
        d, valu_src = matching_profile("*_valu_util.json", mode)
        valu = d["trace_valu_util"] if d else None
    # after the timed region: the same denoiser chain timed over frame-by-frame calls (nothing of the
    # next frame beside or just before it), a labelled extra beside the contract's roofline above
    chain_alone = None
    if pipelined and not banded:
        ds = []
        for _ in range(4):
            r.render_frame(frame, a.spp, params)
            frame += 1
            ds.append(r.timings()["denoise_ms"])
        d_ms = sum(ds) / len(ds)
        ach = B_ALG_PER_PX * band_px / (d_ms * 1e-3) / 1e9
        chain_alone = {"avg_duration_ms": round(d_ms, 4), "achieved": round(ach, 2),
                       "frac": round(ach / HBM_PEAK_GBS, 4), "frames": len(ds),
                       "what": "the denoiser chain of 4 vxpt_render_frame calls after the timed region (HIP "
                               "events on the context stream); in the pipelined run the next frame's first "
                               "pass precedes each chain and the chain measures slower"}
    # the box's practical HBM ceiling ("record the measured copy-kernel bandwidth"): a
    # 1 GiB device-to-device copy, read + write bytes / time, best of 5
    copy_gbs = None
    try:
        src = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:%d" % local)
        dst = torch.empty_like(src)
        best = None
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dst.copy_(src)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        copy_gbs = round(2 * src.numel() / (best * 1e-3) / 1e9, 1)
        del src, dst
    except Exception as e:  # measurement extra only
        print("copy bandwidth not measured: %s" % e, file=sys.stderr)
    depth = r.read("DEPTH")
    hit_frac = float((depth < 1e26).mean())  # scene sanity: fraction of primary rays that hit voxels
    cpu = None
    if rank == 0 and not banded and not a.no_cpu_baseline:
        cpu = cpu_baseline(a, a.cpu_seconds)
    if rank == 0:
        line = {
            "metric": "Mpaths/s @1080p 4spp (+ms/frame, denoiser HBM GB/s vs roofline)",
            "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if banded else "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": ("C2: %dx%d primary-only DDA + sky + G-buffer" % (a.width, a.height) if
                                    a.primary_only else "C3: %dx%d, %d spp full path + ReLAX denoiser" % (
                                        a.width, a.height, a.spp)) + (
                           " on the C1 scene" if a.scene == "c1" else " on the %d^3 world" % a.world),
                       "width": a.width, "height": a.height, "spp": spp,
                       "world": ("C1 scene: 64x32x64 voxels (2x1x2 chunks), Perlin seed 124" if a.scene == "c1" else
                                 "%d^3 voxels, Perlin seed 124" % a.world),
                       "bounces": "%d total / %d diffuse%s" % (
                           a.bounce_limits + ((" (the reference's RayGen.cu:146-147 limits)",) if a.bounce_limits == (3, 1)
                                              else (" (BASELINE.json's '4 bounces' reading; the reference renders 3/1)",)
                                              if a.bounce_limits == (4, 4) else ("",))),
                       "parallelism": ("bands%d (RCCL halo exchange)" % world) if banded else "single GPU",
                       "band_rows": (splits or vxpt.equal_splits(a.height, world)) if banded else None,
                       "band_balance": balance_log,
                       "frame_loop": "vxpt_render_frames (pipelined)" if pipelined else "vxpt_render_frame per step",
                       "tuning": a.tune or "defaults"},
            "mode": mode,
            "roofline": {"bound": "hbm", "kernel": kern, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": round(traffic) if traffic else None, "traffic_source": traffic_src,
                         "alg_bytes_per_launch": alg_bytes, "avg_duration_ms": round(dur_ms, 4)},
            "trace_ms": round(avg_trace, 4), "denoise_ms": round(avg_dn, 4), "timing_source": timing_src,
            "band_diag": band_diag, "band_parity": parity["band_parity"] if parity else None,
            "band_parity_detail": parity, "primary_hit_frac": round(hit_frac, 4),
            # the trace passes over this rank's rows (bands: with their halo exchanges)
            "trace_mpaths_s": round(band_px * spp / (avg_trace * 1e-3) / 1e6, 3),
            "trace_valu_util": valu, "trace_valu_util_source": valu_src, "trace_roofline": trace_roof,
            "roofline_chain_alone": chain_alone,
            "hbm_copy_gbs": copy_gbs,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()
    if parity is not None and not parity["band_parity"]:
        sys.exit(4)


if __name__ == "__main__":
    main()
