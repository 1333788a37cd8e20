"""Multi-GPU band partition (bands.py): the banded render with
its halo exchanges equals the single-band render bit for bit.

CPU: the schedule runs over oracle backends, in one process (LocalExchange)
and across two gloo ranks (DistExchange, the transport the GPU path drives
with RCCL).  GPU: two vxpt contexts on one device, spp = 4.
"""
import os

import numpy as np
import pytest

import bands
import oracle
from band_backends import OracleBand
from golden.make_golden import C1_CAMERA

W, H = 48, 160           # tall frame: two bands of 80 rows >= TRACE_HALO
DN = ([30, 6, 2, 0.5, 0.15, 0.003, 0.01, 0.05, 500000], [1, 1, 1, 1, 1, 1])
P = dict(ta=True, hf=True, hc=True, spatial=True, firefly=True, iters=1)
FRAMES = 3


def _oracle():
    o = oracle.Oracle(W, H)
    o.terrain((2, 1, 2))
    o.set_camera(*C1_CAMERA[:2], fov=C1_CAMERA[2])
    o.set_camera(*C1_CAMERA[:2], fov=C1_CAMERA[2], which=1)
    o.set_sky()
    o.set_denoise_params(*DN)
    return o


def _reference_outputs():
    o = _oracle()
    outs = []
    for f in range(FRAMES):
        o.trace(f)
        o.post_trace()
        o.denoise(f, f + 1)
        outs.append(o.read(21))
    return outs


def test_band_rows_and_plan():
    rows = [bands.band_rows(2160, 8, r) for r in range(8)]
    assert rows[0] == (0, 272) and rows[-1] == (1904, 2160)
    assert all(y0 % 8 == 0 for y0, _ in rows)
    assert sum(y1 - y0 for y0, y1 in rows) == 2160
    for r in range(8):
        for peer, ((sy, sn), (ry, rn)) in bands.halo_plan(rows, r, 72).items():
            back = bands.halo_plan(rows, peer, 72)[r]
            assert (sy, sn) == back[1] and (ry, rn) == back[0]   # what r sends is what peer receives


def test_frame_ops_cover_every_pass():
    ops = list(bands.frame_ops(1, 4, P))
    passes = [o[1] for o in ops if o[0] == "pass"]
    # pass 0 (firefly) writes the world-position plane too; pass 11 alone when the filter is off
    assert passes == [0, 2, 3, 4, 5, 6, 7, 10, 14]
    assert sum(1 for o in ops if o[0] == "trace") == 4
    assert [o[2] for o in ops if o[0] == "trace"] == [2 | 4 | 1024, 2 | 1024, 2 | 1024, 2 | 1024]
    first = list(bands.frame_ops(0, 1, P))
    assert [o[1] for o in first if o[0] == "pass"] == [0, 12, 5, 6, 7, 10, 14]
    nofire = list(bands.frame_ops(1, 1, dict(P, firefly=False)))
    assert [o[1] for o in nofire if o[0] == "pass"] == [11, 2, 3, 4, 5, 6, 7, 10, 14]


def test_oracle_bands_in_process():
    ref = _reference_outputs()
    bands_ = [bands.band_rows(H, 2, r) for r in range(2)]
    backs = [OracleBand(_oracle(), *b) for b in bands_]
    ex = bands.LocalExchange(backs, bands_)
    for f in range(FRAMES):
        bands.run_frame(backs, ex, f, 1, P)
        out = np.concatenate([b.o.read(21)[y0:y1] for b, (y0, y1) in zip(backs, bands_)])
        np.testing.assert_array_equal(out.view(np.uint32), ref[f].view(np.uint32))


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bands_ = [bands.band_rows(H, world, r) for r in range(world)]
        back = OracleBand(_oracle(), *bands_[rank])
        ex = bands.DistExchange(back, bands_, rank)
        outs = []
        for f in range(FRAMES):
            bands.run_frame([back], ex, f, 1, P)
            y0, y1 = bands_[rank]
            outs.append(back.o.read(21)[y0:y1].copy())
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


def test_oracle_bands_gloo_two_ranks():
    import multiprocessing as mp
    import socket
    ref = _reference_outputs()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for f in range(FRAMES):
        out = np.concatenate([res[0][f], res[1][f]])
        np.testing.assert_array_equal(out.view(np.uint32), ref[f].view(np.uint32))


@pytest.mark.gpu
def test_gpu_bands_match_single_context():
    import vxpt
    w, h, spp = 64, 160, 4
    cam = C1_CAMERA

    def make(rows=None):
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_camera(*cam[:2], fov=cam[2], prev=cam)
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    single = make()
    bands_ = [bands.band_rows(h, 2, r) for r in range(2)]
    backs = [bands.GpuBand(make(), y0, y1, p) for y0, y1 in bands_]
    ex = bands.LocalExchange(backs, bands_)
    for f in range(3):
        single.render_frame(f, spp, p)
        bands.run_frame(backs, ex, f, spp, bands.params_dict(p))
        ref = single.read("OUTPUT")
        out = np.concatenate([b.r.read("OUTPUT")[y0:y1] for b, (y0, y1) in zip(backs, bands_)])
        np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n,w,h,splits,tune", [(2, 64, 160, None, None), (8, 640, 640, None, None),
                                               (3, 96, 320, [0, 80, 248, 320], None),
                                               (8, 640, 640, [0, 72, 144, 224, 304, 384, 464, 560, 640], None),
                                               (8, 640, 640, None, "bench"),
                                               (3, 96, 320, [0, 80, 248, 320], "noghost"),
                                               (3, 96, 320, None, "atrous2"), (2, 64, 160, None, "nofix")])
def test_gpu_library_band_schedule_matches_single_context(n, w, h, splits, tune):
    """The library's own band schedule (vxpt_band_link / vxpt_render_frame_linked: the one
    vxpt_band_comm_init runs over RCCL, with device copies between the contexts as the
    transport) equals the single-context render bit for bit; 8 bands simulate the 8-GPU
    partition on one device (bands of 80 rows, wider than the 72-row trace halo).  Uneven
    partitions (vxpt_band_link_rows, the cost-balanced bands of vxpt_band_balance) too, with
    bands as short as the halo itself.  tune "bench": the band contexts run bench.band_tuning's
    schedule (third state set and front stream, straggler walks in 16 pieces); "noghost": the chain
    exchanges after every pass (ghost_rows 0) instead of computing its ghost rows; "atrous2" (two a-trous
    iterations: steps 2..32, ghost margins too deep for the planes' halo, so the per-pass exchange) and
    "nofix" (no history fix: the per-pass schedule too) other denoiser settings."""
    import vxpt
    from bench import band_tuning
    spp = 4
    cam = C1_CAMERA

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_camera(*cam[:2], fov=cam[2], prev=cam)
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    if tune == "atrous2":
        p.atrous_iteration_num = 2
    if tune == "nofix":
        p.enable_history_fix = 0
    single = make()
    rs = [make() for _ in range(n)]
    if tune == "bench":
        t = band_tuning(1920, 1080, n)
        assert t.get("resume_split", 1) > 1
        for r in rs:
            r.set_tuning(**t)
    if tune == "noghost":
        for r in rs:
            r.set_tuning(ghost_rows=0)
    linked = vxpt.LinkedBands(rs, splits)
    rows = [bands.band_rows(h, n, k) for k in range(n)] if splits is None else list(zip(splits[:-1], splits[1:]))
    for f in range(3):
        single.render_frame(f, spp, p)
        linked.render_frame(f, spp, p)
        ref = single.read("OUTPUT")
        out = np.concatenate([r.read("OUTPUT")[y0:y1] for r, (y0, y1) in zip(rs, rows)])
        np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n,w,h,variant", [(2, 96, 160, "yaml"), (2, 96, 160, "wide_bloom_flare"),
                                           (8, 640, 640, "yaml")])
def test_gpu_band_postprocess_matches_single_context(n, w, h, variant):
    """A banded frame's post-process (vxpt_postprocess_linked: the denoiser output's 1-row halo,
    the histogram + sun flag summed over the bands, the bloom's halo; the RCCL path differs
    only in the transport) equals the single-context post-process bit for bit over 3 frames
    (the auto exposure's state carries across frames)."""
    import vxpt
    cam = C1_CAMERA

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_camera(*cam[:2], fov=cam[2], prev=cam)
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    single = make()
    pp = single.post_params()
    if variant == "wide_bloom_flare":  # the 2-pass bloom (radius past the LDS apron), lens flare, vignette
        pp.bloom_radius, pp.bloom_threshold, pp.enable_lens_flare, pp.enable_vignette = 10.0, 0.05, 1, 1
    rs = [make() for _ in range(n)]
    linked = vxpt.LinkedBands(rs)
    rows = [bands.band_rows(h, n, k) for k in range(n)]
    for f in range(3):
        single.render_frame(f, 1, p)
        linked.render_frame(f, 1, p)
        single.postprocess(pp, 16.0)
        linked.postprocess(pp, 16.0)
        ref = single.read("FRAME")
        out = np.concatenate([r.read("FRAME")[y0:y1] for r, (y0, y1) in zip(rs, rows)])
        np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_library_band_functions_match_bands_py():
    """vxpt_band_rows / vxpt_halo_plan (pure host functions of the C ABI) equal bands.py's."""
    import vxpt
    for H in (160, 640, 1080, 2160):
        for n in (1, 2, 3, 8):
            rows = [bands.band_rows(H, n, r) for r in range(n)]
            for r in range(n):
                assert vxpt.band_rows(H, n, r) == rows[r]
                for depth in (0, 2, 34, 72, 91):
                    assert vxpt.halo_plan(H, n, r, depth) == bands.halo_plan(rows, r, depth), (H, n, r, depth)


def _check_splits(s, h, n):
    assert len(s) == n + 1 and s[0] == 0 and s[-1] == h
    assert all(b - a >= 72 for a, b in zip(s[:-1], s[1:])), s
    assert all(v % 8 == 0 for v in s[1:-1]), s


def test_band_balance_equalises_a_cost_profile():
    """vxpt_band_balance: from the band times of a partition, boundaries whose bands cost alike.
    A synthetic per-row cost (expensive horizon rows above cheap ground rows, as in the C3 view)
    measured over the equal bands, then over each proposed partition: three rounds bring the
    slowest band within 6% of the mean (equal bands: 25-60% above it)."""
    import vxpt
    for h, n in ((1080, 2), (1080, 4), (1080, 8), (2160, 8)):
        y = np.arange(h) + 0.5
        row_cost = 0.4 + np.exp(-((y / h - 0.3) / 0.3) ** 2)
        measure = lambda s: [float(row_cost[a:b].sum()) for a, b in zip(s[:-1], s[1:])]  # noqa: E731
        s = vxpt.equal_splits(h, n)
        t = measure(s)
        first = max(t) / np.mean(t)
        cost = None
        for _ in range(3):
            s, cost = vxpt.band_balance(h, s, t, cost)
            _check_splits(s, h, n)
            t = measure(s)
        assert first > 1.2 and max(t) / np.mean(t) < 1.06, (h, n, first, max(t) / np.mean(t), s)


def test_band_balance_keeps_uniform_costs_and_rejects_bad_partitions():
    import vxpt
    s, cost = vxpt.band_balance(1080, vxpt.equal_splits(1080, 4), [1.0] * 4)
    _check_splits(s, 1080, 4)
    assert max(abs(a - b) for a, b in zip(s, [0, 272, 544, 816, 1080])) <= 8
    assert cost.shape == (135,) and np.allclose(cost.sum(), 4.0, rtol=1e-5)
    # a band that costs nothing still keeps the halo's 72 rows
    s, _ = vxpt.band_balance(640, vxpt.equal_splits(640, 8), [0.0] * 7 + [10.0])
    _check_splits(s, 640, 8)
    for bad in ([0, 100, 200], [0, 64, 200], [8, 100, 200], [0, 100, 208]):
        with pytest.raises(vxpt.VxptError):
            vxpt.band_balance(200, bad, [1.0, 1.0])
    with pytest.raises(vxpt.VxptError):
        vxpt.band_balance(200, [0, 96, 200], [1.0, -1.0])


class _TimedBand:
    """A stand-in renderer for bench.balance_bands: a frame of band [y0, y1) takes the synthetic
    cost of its rows in wall time (20 ms for a whole 1080-row frame, rows near the top 3x the rest: long
    enough that scheduling noise on a loaded host stays a few per cent of a band's time)."""
    def __init__(self):
        self.y0, self.y1 = 0, 1080

    def set_band(self, y0, y1):
        self.y0, self.y1 = y0, y1

    def render_frames(self, f0, n, spp, params):
        import time
        y = np.arange(self.y0, self.y1)
        time.sleep(n * float(np.where(y < 360, 3.0, 1.0).sum()) * 20e-3 / 1800.0)

    def sync(self):
        pass

    def close(self):
        pass


def _balance_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        class A:
            height, spp, primary_only = 1080, 4, False
        splits, log = bench.balance_bands(A, _TimedBand, None, world, rank, dist)
        q.put((rank, splits, log))
    finally:
        dist.destroy_process_group()


def test_bench_band_balance_gloo_two_ranks():
    """bench.balance_bands over two gloo ranks (the N>1 bench's pre-run step): both ranks time their
    band, share the times and arrive at the same boundaries, which move the split towards the
    expensive top rows (cost 3 per row above row 360, 1 below: equal cost at row 300)."""
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_balance_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (sp, log) for r, sp, log in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    splits, log = res[0]
    assert log[0]["band_rows"] == [0, 544, 1080] and len(log) == 4
    assert splits[0] == 0 and splits[2] == 1080 and 280 <= splits[1] <= 320, splits  # 544 -> ~384 -> ~312 -> ~304


def _turn(d, yaw_deg, pitch_deg):
    import math
    y = math.atan2(d[0], d[2]) + math.radians(yaw_deg)
    p = math.asin(max(-1.0, min(1.0, d[1]))) + math.radians(pitch_deg)
    return (math.sin(y) * math.cos(p), math.sin(p), math.cos(y) * math.cos(p))


def test_band_halo_rows_follow_the_camera():
    """vxpt_band_halo_rows: the static depths for an unmoved camera, deeper halos as the camera turns
    further, refusal for a translation or a turn past the band height."""
    import vxpt
    cam = C1_CAMERA
    assert vxpt.band_halo_rows(cam, cam, 640, 640, 8) == (72, 2)
    assert vxpt.band_halo_rows(cam, cam, 640, 640, 1) == (72, 2)
    moved = ((cam[0][0] + 0.1, cam[0][1], cam[0][2]), cam[1], cam[2])
    assert vxpt.band_halo_rows(moved, cam, 640, 640, 2) is None
    assert vxpt.band_halo_rows(moved, cam, 640, 640, 2, near=0.0) is None
    last = (72, 2)
    for pitch in (0.2, 0.5, 1.0, 1.5):
        got = vxpt.band_halo_rows((cam[0], _turn(cam[1], 0.0, pitch), cam[2]), cam, 640, 640, 2)
        assert got is not None and got[0] >= last[0] and got[1] >= last[1] and got[1] > 2, (pitch, got)
        assert got[0] >= 64 + got[1] - 1
        last = got
    # 8 bands of 80 rows: a 3-degree pitch needs more than a band
    assert vxpt.band_halo_rows((cam[0], _turn(cam[1], 0.0, 3.0), cam[2]), cam, 640, 640, 8) is None
    assert vxpt.band_halo_rows((cam[0], _turn(cam[1], 0.0, 3.0), cam[2]), cam, 640, 640, 2) is not None


def test_band_halo_rows_bound_a_translation():
    """vxpt_band_halo_rows_near: a translating camera gets halos from the hit-distance bound -- deeper
    for nearer surfaces and longer moves, the rotation's depths as the bound goes to infinity, refused
    when the bound is too small for the bands; every reprojected row of a hit at or beyond the bound
    (sampled pixels, random distances) lies within the returned history depth."""
    import vxpt
    cam = C1_CAMERA
    w, h = 640, 640
    up = ((cam[0][0], cam[0][1] + 0.05, cam[0][2]), cam[1], cam[2])
    far = vxpt.band_halo_rows(up, cam, w, h, 2, near=1e6)
    # the rotation's computed depths (margins included) for an unturned camera
    assert far[0] == 72 and far[1] <= 5
    last = far
    for near in (40.0, 10.0, 3.0, 1.0):
        got = vxpt.band_halo_rows(up, cam, w, h, 2, near=near)
        assert got is not None and got[0] >= last[0] and got[1] >= last[1], (near, got)
        last = got
    assert last[1] > 2
    longer = ((cam[0][0], cam[0][1] + 0.5, cam[0][2]), cam[1], cam[2])
    assert vxpt.band_halo_rows(longer, cam, w, h, 2, near=1.0)[1] > last[1]
    assert vxpt.band_halo_rows(longer, cam, w, h, 8, near=0.2) is None
    # the bound holds for sampled hits: project them with the camera model of band_halo_rows
    near, (tr, hr) = 3.0, vxpt.band_halo_rows(up, cam, w, h, 2, near=3.0)
    rng = np.random.default_rng(3)

    def basis(c):
        d = np.asarray(c[1], np.float64)
        d /= np.linalg.norm(d)
        right = np.cross(d, [0.0, 1.0, 0.0])
        right /= np.linalg.norm(right)
        upv = np.cross(right, d)
        t = np.tan(np.radians(c[2]) / 2)
        return d, right * t * w / h, upv * t

    cd, cr, cu = basis(up)
    pd, pr, pu = basis(cam)
    y0, y1 = bands.band_rows(h, 2, 0)
    for _ in range(4000):
        px, py = rng.uniform(0, w), rng.uniform(y0, y1)
        ray = cd + cr * (2 * px / w - 1) - cu * (2 * py / h - 1)
        ray /= np.linalg.norm(ray)
        hit = np.asarray(up[0]) + ray * near * (1 + rng.exponential(2.0))
        v = hit - np.asarray(cam[0])
        z = v @ pd
        row = (1 - (v @ pu) / np.linalg.norm(pu) ** 2 / z) * h / 2
        assert row < y1 + hr, (px, py, row)


def _near_bound(o):
    """nearest_surface restated over the oracle's voxels, brute force: the distance from the camera
    to the nearest non-air cell grown by one cell"""
    cx, cy, cz = o.chunks
    ids = o.voxels().reshape(cz * cx * cy, 32, 32, 32)  # chunk, y, z, x
    ch, yy, zz, xx = np.nonzero(ids)
    x = (ch % cx) * 32 + xx
    z = ((ch // cx) % cz) * 32 + zz
    y = (ch // (cx * cz)) * 32 + yy

    def gap(p, lo):
        a, b = lo - 1.0, lo + 2.0
        return np.where(p < a, a - p, np.where(p > b, p - b, 0.0))

    def near(pos):
        d = np.sqrt(gap(pos[0], x) ** 2 + gap(pos[1], y) ** 2 + gap(pos[2], z) ** 2)
        return float(min(d.min(), 62.0))
    return near


def test_oracle_bands_follow_a_translating_camera():
    """A camera that moves (and turns) between frames: halo depths from vxpt_band_halo_rows_near with
    the world's nearest-surface bound (as vxpt_render_frame computes it) render the oracle's two bands
    bit for bit like one band."""
    import vxpt
    bands_ = [bands.band_rows(H, 2, r) for r in range(2)]
    single = _oracle()
    backs = [OracleBand(_oracle(), *b) for b in bands_]
    ex = bands.LocalExchange(backs, bands_)
    near_of = _near_bound(single)
    moves = [((0, 0, 0), 0), ((0, 0.15, 0), 0), ((0.1, -0.1, -0.1), 1.0), ((0, 0, 0), 0)]
    pos, d = list(C1_CAMERA[0]), C1_CAMERA[1]
    prev, prev_halo, deep = C1_CAMERA, (bands.TRACE_HALO, 2), 0
    for f, (dp, pitch) in enumerate(moves):
        pos = [pos[k] + dp[k] for k in range(3)]
        d = _turn(d, 0.0, pitch)
        cur = (tuple(pos), d, C1_CAMERA[2])
        for o in [single] + [b.o for b in backs]:
            o.set_camera(*cur[:2], fov=cur[2])
            o.set_camera(*prev[:2], fov=prev[2], which=1)
        halo = vxpt.band_halo_rows(cur, prev, W, H, 2, near=near_of(pos))
        assert halo is not None, f
        deep += halo[1] > 2
        single.trace(f)
        single.post_trace()
        single.denoise(f, f + 1)
        bands.run_frame(backs, ex, f, 1, P, halo, prev_halo)
        out = np.concatenate([b.o.read(21)[y0:y1] for b, (y0, y1) in zip(backs, bands_)])
        np.testing.assert_array_equal(out.view(np.uint32), single.read(21).view(np.uint32), err_msg="frame %d" % f)
        prev, prev_halo = cur, halo
    assert deep >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("n,w,h,turns", [
    (2, 96, 320, [(0, 0), (2, 0.8), (0, 3), (0, 2), (1, 1)]),
    # a 10-degree pitch: history halo 53 rows, deeper than the ghost rows' 40 (the clamp's histories exchanged)
    (2, 96, 320, [(0, 0), (0, 10), (0, 2)]),
    (8, 640, 640, [(0, 0), (1, 0.3), (0.5, 0.5), (1.5, 0.4), (0, 1.0)])])
def test_gpu_linked_bands_follow_a_turning_camera(n, w, h, turns):
    """A camera that yaws / pitches between frames: the banded frame deepens its halos
    (vxpt_band_halo_rows: the reprojected rows of the ReSTIR temporal taps and the history taps)
    and stays bit-exact against one context; the end-of-frame gather leaves the whole frame in
    band 0; a turn past the band height is refused."""
    import vxpt
    spp = 2
    cam = C1_CAMERA

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    single = make()
    rs = [make() for _ in range(n)]
    linked = vxpt.LinkedBands(rs)
    rows = [bands.band_rows(h, n, k) for k in range(n)]
    d, prev, deep = cam[1], cam, 0
    for f, (dy, dp) in enumerate(turns):
        d = _turn(d, dy, dp)
        cur = (cam[0], d, cam[2])
        halo = vxpt.band_halo_rows(cur, prev, w, h, n)
        assert halo is not None
        deep += halo != (72, 2)
        for r in [single] + rs:
            r.set_camera(*cur[:2], fov=cur[2], prev=prev)
        single.render_frame(f, spp, p)
        linked.render_frame(f, spp, p)
        ref = single.read("OUTPUT")
        out = np.concatenate([r.read("OUTPUT")[y0:y1] for r, (y0, y1) in zip(rs, rows)])
        np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32), err_msg="frame %d" % f)
        linked.gather("OUTPUT", 0)
        np.testing.assert_array_equal(rs[0].read("OUTPUT").view(np.uint32), ref.view(np.uint32))
        prev = cur
    assert deep >= 2
    far = (cam[0], _turn(d, 0.0, 30.0), cam[2])
    for r in rs:
        r.set_camera(*far[:2], fov=far[2], prev=prev)
    with pytest.raises(vxpt.VxptError):
        linked.render_frame(len(turns), spp, p)


@pytest.mark.gpu
def test_gpu_nearest_surface_matches_restatement():
    """vxpt_nearest_surface over the host mirror of the world equals the brute-force restatement over
    the oracle's voxels (nearest non-air cell grown by one cell, capped at 62) at random positions in
    and around the C1 world, before and after a block edit next to the probe."""
    import vxpt
    r = vxpt.Renderer(32, 32)
    r.load_settings()
    r.generate_terrain((2, 1, 2))
    o = oracle.Oracle(8, 8)
    o.terrain((2, 1, 2))
    near_of = _near_bound(o)
    rng = np.random.default_rng(11)
    pts = rng.uniform([-20.0, -10.0, -20.0], [84.0, 60.0, 84.0], size=(200, 3))
    for p in pts:
        assert abs(r.nearest_surface(p) - near_of(p)) < 1e-4, p
    # a block placed in the air beside a probe point: the bound drops to it
    p = (35.6, 29.3, 42.1)  # ~17.6 above the terrain there
    before = r.nearest_surface(p)
    r.set_block(35, 31, 42, 1)
    after = r.nearest_surface(p)
    assert after < before and abs(after - 0.7) < 1e-4, (before, after)
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,w,h", [(2, 96, 320), (8, 640, 640)])
def test_gpu_linked_bands_follow_a_translating_camera(n, w, h):
    """A camera that moves (and turns) between frames: the banded frame takes its halo depths from
    the world's nearest-surface bound (vxpt_nearest_surface, equal to the restatement over the
    oracle's voxels) and stays bit-exact against one context; a move too long for the bands is
    refused."""
    import vxpt
    spp = 2

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_sky()
        return r

    o = oracle.Oracle(8, 8)
    o.terrain((2, 1, 2))
    near_of = _near_bound(o)
    p = vxpt.DenoiseParams.defaults()
    single = make()
    rs = [make() for _ in range(n)]
    linked = vxpt.LinkedBands(rs)
    rows = [bands.band_rows(h, n, k) for k in range(n)]
    moves = [((0, 0, 0), 0), ((0, 0.02, 0), 0), ((0.02, -0.02, -0.02), 0.3), ((0, 0, 0.03), 0), ((0, 0, 0), 0)]
    pos, d = list(C1_CAMERA[0]), C1_CAMERA[1]
    prev, deep = C1_CAMERA, 0
    for f, (dp, pitch) in enumerate(moves):
        pos = [pos[k] + dp[k] for k in range(3)]
        d = _turn(d, 0.0, pitch)
        cur = (tuple(pos), d, C1_CAMERA[2])
        assert abs(single.nearest_surface(pos) - near_of(pos)) < 1e-4
        halo = vxpt.band_halo_rows(cur, prev, w, h, n, near=single.nearest_surface(pos))
        assert halo is not None, f
        deep += halo[1] > 2
        for r in [single] + rs:
            r.set_camera(*cur[:2], fov=cur[2], prev=prev)
        single.render_frame(f, spp, p)
        linked.render_frame(f, spp, p)
        ref = single.read("OUTPUT")
        out = np.concatenate([r.read("OUTPUT")[y0:y1] for r, (y0, y1) in zip(rs, rows)])
        np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32), err_msg="frame %d" % f)
        prev = cur
    assert deep >= 2
    far = ((pos[0], pos[1] + 2.0, pos[2]), d, C1_CAMERA[2])
    for r in rs:
        r.set_camera(*far[:2], fov=far[2], prev=prev)
    with pytest.raises(vxpt.VxptError):
        linked.render_frame(len(moves), spp, p)


def _oracle_turning(turns, halos_from_library):
    """Banded (2 oracle bands, LocalExchange) and single-band oracle renders of a camera turning
    between frames; the banded schedule's halo depths come from the library's vxpt_band_halo_rows
    (or stay static).  Returns the per-frame outputs of both."""
    import vxpt
    bands_ = [bands.band_rows(H, 2, r) for r in range(2)]
    single = _oracle()
    backs = [OracleBand(_oracle(), *b) for b in bands_]
    ex = bands.LocalExchange(backs, bands_)
    d, prev, prev_halo = C1_CAMERA[1], C1_CAMERA, (bands.TRACE_HALO, 2)
    outs = []
    for f, (dy, dp) in enumerate(turns):
        d = _turn(d, dy, dp)
        cur = (C1_CAMERA[0], d, C1_CAMERA[2])
        for o in [single] + [b.o for b in backs]:
            o.set_camera(*cur[:2], fov=cur[2])
            o.set_camera(*prev[:2], fov=prev[2], which=1)
        halo = vxpt.band_halo_rows(cur, prev, W, H, 2) if halos_from_library else (bands.TRACE_HALO, 2)
        assert halo is not None
        single.trace(f)
        single.post_trace()
        single.denoise(f, f + 1)
        bands.run_frame(backs, ex, f, 1, P, halo, prev_halo)
        out = np.concatenate([b.o.read(21)[y0:y1] for b, (y0, y1) in zip(backs, bands_)])
        outs.append((single.read(21), out, halo))
        prev, prev_halo = cur, halo
    return outs


def test_oracle_bands_follow_a_turning_camera():
    """The band schedule with the library's camera-aware halo depths (vxpt_band_halo_rows, topped
    up at the start of a frame) renders a pitching camera bit for bit like one band; the static
    depths do not -- so the computed depths are what makes it exact."""
    turns = [(0, 0), (0, 3), (1, -3), (0, 0)]
    good = _oracle_turning(turns, True)
    assert any(h != (bands.TRACE_HALO, 2) for _, _, h in good)
    for f, (ref, out, _) in enumerate(good):
        np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32), err_msg="frame %d" % f)
    static = _oracle_turning(turns, False)
    assert any(not np.array_equal(out.view(np.uint32), ref.view(np.uint32)) for ref, out, _ in static)


@pytest.mark.gpu
def test_gpu_c4_eight_bands_4k_c3_world():
    """BASELINE config C4's workload on one device: 3840x2160, 4 spp, the C3 256^3 world and camera
    (bench.py's scene), split into 8 linked bands of 272 rows (8-row aligned; the last 256) -- the
    schedule vxpt_band_comm_init runs over RCCL, with device copies as the transport.  After each
    of 3 frames the gathered denoiser output and post-processed frame (vxpt_band_gather_linked into
    band 0) equal one context's render bit for bit.  Footprint: 9 contexts with full-frame 4K planes
    (~6 GB each) + wavefront state for their rows (two sets) -- ~75 GB of the device's 288."""
    import vxpt
    from bench import C1_DIR, scene_args

    class A:
        world = 256
        scene = "c3"

    chunks, hs, fd, gy, pos = scene_args(A)
    w, h, spp, n = 3840, 2160, 4, 8

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain(chunks, height_scale=hs, freq_den=fd, global_y=gy)
        r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    single = make()
    rs = [make() for _ in range(n)]
    try:
        linked = vxpt.LinkedBands(rs)
        rows = [bands.band_rows(h, n, k) for k in range(n)]
        assert rows[0] == (0, 272) and rows[-1] == (1904, 2160)
        pp = single.post_params()
        for f in range(3):
            single.render_frame(f, spp, p)
            linked.render_frame(f, spp, p)
            single.postprocess(pp, 16.0)
            linked.postprocess(pp, 16.0)
            for name in ("OUTPUT", "FRAME"):
                linked.gather(name, 0)
                got, ref = rs[0].read(name), single.read(name)
                assert np.isfinite(ref).all()
                np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32), err_msg="frame %d %s" % (f, name))
        hit = (single.read("DEPTH") < 1e26).mean()
        assert 0.5 < hit < 0.9, hit  # the C3 camera sees terrain and sky
    finally:
        single.close()
        for r in rs:
            r.close()


@pytest.mark.gpu
def test_gpu_rccl_one_rank_communicator_matches_plain_context():
    """vxpt_band_comm_init with a one-rank communicator: ncclCommInitRank, the banded frame over the
    communicator (its halo groups have no peer), the post-process histogram ncclAllReduce and
    vxpt_band_gather run on one device -- RCCL executing in the library -- and equal a plain
    context bit for bit over 3 frames (OUTPUT, FRAME)."""
    import vxpt
    w, h, spp = 96, 80, 4
    cam = C1_CAMERA

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_camera(*cam[:2], fov=cam[2], prev=cam)
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    a, b = make(), make()
    try:
        b.band_comm_init(vxpt.band_comm_id(), 1, 0)
        for f in range(3):
            a.render_frame(f, spp, p)
            b.render_frame(f, spp, p)
            a.postprocess()
            b.postprocess()
            b.band_gather("OUTPUT")
            for name in ("OUTPUT", "FRAME"):
                np.testing.assert_array_equal(a.read(name).view(np.uint32), b.read(name).view(np.uint32),
                                              err_msg="frame %d %s" % (f, name))
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_gpu_rccl_one_rank_render_frames_matches_plain_context():
    """vxpt_render_frames on a context with a (one-rank) communicator enqueues its banded frames back
    to back with one sync at the end: the same OUTPUT bit for bit as a plain context's run, and
    frame / trace / denoiser timings from the run's events."""
    import vxpt
    w, h, spp = 96, 80, 4
    cam = C1_CAMERA

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_camera(*cam[:2], fov=cam[2], prev=cam)
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    a, b = make(), make()
    try:
        b.band_comm_init(vxpt.band_comm_id(), 1, 0)
        a.render_frames(0, 4, spp, p)
        b.render_frames(0, 4, spp, p)
        np.testing.assert_array_equal(a.read("OUTPUT").view(np.uint32), b.read("OUTPUT").view(np.uint32))
        t = b.timings()
        assert t["frame_ms"] > 0 and t["trace_ms"] > 0 and t["denoise_ms"] > 0, t
        # the band instrumentation of the same run: every frame's spans, its exchange groups (a single
        # rank has no neighbour: nothing sent), results unchanged
        b.band_stats_enable(True)
        a.render_frames(4, 3, spp, p)
        b.render_frames(4, 3, spp, p)
        st = b.band_stats()
        np.testing.assert_array_equal(a.read("OUTPUT").view(np.uint32), b.read("OUTPUT").view(np.uint32))
        assert st["frames"] == 3 and st["groups"] >= 3 * 5 and st["groups_ordered"] < st["groups"], st
        assert st["bytes_up"] == 0 and st["bytes_down"] == 0, st
        assert st["trace_ms"] > 0 and st["denoise_ms"] > 0 and st["exchange_ms"] >= 0, st
        assert (st["row_begin"], st["row_end"]) == (0, h), st
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_gpu_band_stats_linked_bands():
    """vxpt_band_stats over linked contexts (the multi-GPU run's self-description): every frame's
    trace and denoiser spans, the exchange groups, and the bytes each band sends a neighbour -- the
    halo plan's rows of every exchanged buffer, the same both ways across a border; results unchanged."""
    import vxpt
    w, h, spp, n = 96, 240, 4, 3
    cam = C1_CAMERA

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_camera(*cam[:2], fov=cam[2], prev=cam)
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    single = make()
    rs = [make() for _ in range(n)]
    linked = vxpt.LinkedBands(rs)
    rows = [bands.band_rows(h, n, k) for k in range(n)]
    for r in rs:
        r.band_stats_enable(True)
    for f in range(3):
        single.render_frame(f, spp, p)
        linked.render_frame(f, spp, p)
    out = np.concatenate([r.read("OUTPUT")[y0:y1] for r, (y0, y1) in zip(rs, rows)])
    np.testing.assert_array_equal(out.view(np.uint32), single.read("OUTPUT").view(np.uint32))
    st = [r.band_stats() for r in rs]
    for k, s in enumerate(st):
        assert s["frames"] == 3 and s["groups"] >= 3 * 8, s
        assert s["trace_ms"] > 0 and s["denoise_ms"] > 0 and s["exchange_ms"] > 0, s
        assert (s["row_begin"], s["row_end"]) == rows[k], s
    assert st[0]["bytes_up"] == 0 and st[-1]["bytes_down"] == 0
    for k in range(n - 1):  # a border's rows move the same way both ways (equal band heights)
        assert st[k]["bytes_down"] > 0 and st[k]["bytes_down"] == st[k + 1]["bytes_up"], (k, st)
    for r in rs:
        r.close()
    single.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,spp,tune", [(2, 160, 1, None), (2, 160, 4, None), (3, 240, 4, None),
                                          (3, 240, 4, dict(chain_gate=0)), (2, 160, 1, dict(chain_gate=0)),
                                          (3, 240, 4, dict(chain_gate=0, state_sets=3, front_streams=3))])
def test_gpu_linked_render_frames_pipelined_matches_frame_calls(n, h, spp, tune):
    """The banded vxpt_render_frames schedule (band_frame's pipe: the next frame's first pass-halves
    enqueued beside the last second half and its exchange, the chain after them, the later first halves
    gated on the host) run with neighbours: vxpt_render_frames_linked over n linked bands x 4 frames
    equals n x 4 vxpt_render_frame_linked calls and one whole-frame context, bit for bit.  Then bench.py's
    own self-check of a banded run (band_parity): the OUTPUT gathered at the root band against
    bench.single_context_frames of the same frame sequence -- true, and false with the rows named when
    one band's row is disturbed.  tune chain_gate 0: the later first halves not gated behind the previous
    frame's chain (bench.band_tuning's schedule; at spp 1 the library keeps the gate)."""
    import vxpt
    from bench import band_parity, single_context_frames
    w, frames = 96, 4
    cam = C1_CAMERA

    def make():
        r = vxpt.Renderer(w, h)
        r.load_settings()
        r.generate_terrain((2, 1, 2))
        r.set_camera(*cam[:2], fov=cam[2], prev=cam)
        r.set_sky()
        return r

    p = vxpt.DenoiseParams.defaults()
    rows = [bands.band_rows(h, n, k) for k in range(n)]
    piped = [make() for _ in range(n)]
    calls = [make() for _ in range(n)]
    if tune:
        for r in piped:
            r.set_tuning(**tune)
    try:
        lp, lc = vxpt.LinkedBands(piped), vxpt.LinkedBands(calls)
        lp.render_frames(0, frames, spp, p)
        for f in range(frames):
            lc.render_frame(f, spp, p)
        for name in ("OUTPUT", "ILLUM", "PREV_ILLUM", "HIST_LEN"):
            for k, (y0, y1) in enumerate(rows):
                np.testing.assert_array_equal(piped[k].read(name)[y0:y1].view(np.uint32),
                                              calls[k].read(name)[y0:y1].view(np.uint32),
                                              err_msg="%s band %d" % (name, k))
        lp.gather("OUTPUT", 0)
        single = single_context_frames(make, frames, spp, p)
        try:
            ref = single.read("OUTPUT")
        finally:
            single.close()
        res = band_parity(piped[0].read("OUTPUT"), ref)
        assert res == {"band_parity": True, "mismatched_px": 0}, res
        bad = piped[0].read("OUTPUT")
        y = rows[-1][0] + 3  # a row of the last band, as gathered at the root
        bad[y, 5, 0] = np.nextafter(bad[y, 5, 0], np.float32(np.inf))
        res = band_parity(bad, ref)
        assert not res["band_parity"] and res["mismatched_px"] == 1 and res["mismatched_rows"] == [y, y], res
    finally:
        for r in piped + calls:
            r.close()


def test_band_parity_helper_and_watchdog():
    """bench.band_parity on host arrays (bit-exact per pixel, every channel; -0.0 vs 0.0 differs), and the
    bench watchdog ending a process whose armed section outlives its limit with status 5."""
    import subprocess
    import sys
    from bench import REPO, band_parity
    a = np.random.default_rng(3).random((16, 8, 4), dtype=np.float32)
    assert band_parity(a, a.copy()) == {"band_parity": True, "mismatched_px": 0}
    b = a.copy()
    b[2, 1, 3] = -0.0 if a[2, 1, 3] == 0 else np.float32(0.0)
    b[9, 7, :] = np.float32(-0.0)
    r = band_parity(a, b)
    assert not r["band_parity"] and r["mismatched_px"] == 2 and r["mismatched_rows"] == [2, 9], r
    z = np.zeros((4, 4, 4), np.float32)
    assert not band_parity(z, -z)["band_parity"]
    assert band_parity(a, a[:8])["band_parity"] is False
    code = ("import sys, time; sys.path.insert(0, %r); import bench; w = bench.Watchdog(1); "
            "w.arm(0.5, 'a stuck frame'); time.sleep(30)") % REPO
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 5 and "a stuck frame" in p.stderr, (p.returncode, p.stderr)
