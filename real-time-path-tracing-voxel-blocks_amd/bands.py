"""Screen-band partition of the offline render across GPUs.

Each rank owns rows [y0, y1) of the frame (8-row aligned) and traces and
denoises only those rows into full-frame buffers.  Every pass that reads a
neighbourhood is preceded by an exchange of the rows it reads outside the
band, taken from the ranks that own them -- so the banded render is the
single-GPU render, bit for bit.  The schedule below mirrors one
OfflineBackend::renderFrame (vxpt_render_frame / do_denoise in vxpt_host.cpp)
with the exchanges inserted:

  trace pass s      -> G-buffer + reservoirs of that pass, TRACE_HALO rows:
                       ReSTIR temporal taps of the next pass read the previous
                       pass's surfaces and reservoirs within a 64-pixel disk
                       around the reprojected pixel (Restir.h:348-381)
  firefly filter    -> reservoirs (next frame's taps) and radiance (HC 5x5)
  temporal accum.   -> ping for HistoryFix: 5x5 taps at radius 2^(4-h)+1 <= 17
                       (HistoryFix.h:12-17) -> 34 rows; pong for clamping: 2
  history clamping  -> the histories the next frame reprojects into (bicubic: 2)
  a-trous passes    -> their output for the next step s: s rows (+ s/4 jitter above 4)

The rows are moved by a transport: DistExchange (torch.distributed: RCCL over
xGMI on GPUs, gloo on CPU) or LocalExchange (bands of one process; tests).
Bands must be at least TRACE_HALO rows tall.  A camera that turns between
frames needs deeper halos: pass run_frame the depths vxpt.band_halo_rows gives
for the frame's camera pair (and the previous frame's), as the library's own
schedule (vxpt_render_frame with a communicator, vxpt_render_frame_linked) does.  (The library's
own chain computes the history clamp's and the a-trous steps' out-of-band rows itself -- its ghost
rows, tuning ghost_rows -- instead of exchanging after each of those passes; this host-driven schedule
keeps one exchange per pass.  Both are the single-GPU render bit for bit.)
"""
import numpy as np

TRACE_HALO = 72
GBUF = ["DEPTH", "NORMAL_ROUGH", "GEO_NORMAL_THIN", "ALBEDO", "MATERIAL", "MAT_PARAM"]
RES = ["RES_EVEN", "RES_ODD"]
HISTORY = ["PREV_ILLUM", "PREV_FAST", "PREV_HIST_LEN"]

ACCUMULATE, ACCUM_FIRST = 2, 4


def band_rows(H, world, rank):
    """Rows of `rank`: equal 8-row-aligned bands, the last one takes the rest."""
    per = -(-H // (8 * world)) * 8
    y0 = min(H, rank * per)
    return y0, min(H, y0 + per)


def atrous_rows(step):
    """Rows an a-trous pass of `step` reads beyond its pixel (Atrous.h:79-84 jitter above step 4)."""
    return step + (step // 4 if step > 4 else 0)


# the previous pass's G-buffer as the next trace reads it ("PREV:<name>"): the library's last slot
# (the same buffer as <name>), the oracle's Prev* copies
PREV_GBUF = ["PREV:" + n for n in GBUF]


def frame_ops(frame, spp, p, halo=(TRACE_HALO, 2), prev_halo=(TRACE_HALO, 2)):
    """Operations of one banded frame.  p: dict with the denoiser switches
    (ta, hf, hc, spatial, firefly, iters).  halo: (trace rows, history rows) for this frame's
    camera motion (vxpt.band_halo_rows); prev_halo: the depths the previous frame exchanged --
    deeper halos are topped up before the first pass.  Yields ("trace", it, flags),
    ("post_trace",), ("pass", id, arg, arg2), ("exchange", [buffers], rows)."""
    it0 = frame * spp
    trace_rows, hist_rows = halo
    if frame > 0 and (trace_rows > prev_halo[0] or hist_rows > prev_halo[1]):
        yield ("exchange", PREV_GBUF + [RES[(it0 - 1) & 1]], trace_rows)
        yield ("exchange", HISTORY, hist_rows)
    for s in range(spp):
        flags = 0 if spp == 1 else (ACCUMULATE | (ACCUM_FIRST if s == 0 else 0) | (spp << 8))
        yield ("trace", it0 + s, flags)
        yield ("exchange", GBUF + [RES[(it0 + s) & 1]], trace_rows)
        yield ("post_trace",)
    yield ("exchange", ["ILLUM"], 2)
    it = it0 + spp
    used = it - 1 if it > 0 else 0
    if p["firefly"]:
        # the firefly pass writes the world-position plane too (pass 11 alone otherwise)
        yield ("pass", 0, used & 1, 0)
        yield ("exchange", [RES[used & 1]], trace_rows)
        yield ("exchange", ["ILLUM"], 2)
    else:
        yield ("pass", 11, 0, 0)
    if frame == 0:
        yield ("pass", 12, 0, 0)
        yield ("exchange", HISTORY, hist_rows)
    fin = 0
    if p["ta"] and frame > 0:
        yield ("pass", 2, 0, 0)
        yield ("exchange", ["PING"], 34)
        yield ("exchange", ["PONG"], 2)
        fin = 1
        if p["hf"]:
            yield ("pass", 3, 0, 0)
            yield ("exchange", ["PONG"], 2)
            fin = 2
        if p["hc"]:
            yield ("pass", 4, 0, 0)
            yield ("exchange", HISTORY, hist_rows)
            fin = 3
    out_done = False
    if p["spatial"]:
        yield ("pass", 5, 0, 0)
        yield ("exchange", ["PING"], atrous_rows(2))
        fin = 1
        if p["iters"] > 0:
            idx, step = 1, 2
            while idx < 2 * p["iters"]:
                yield ("pass", 6, step, it)
                idx += 1
                step = 1 << idx
                yield ("exchange", ["PONG"], atrous_rows(step))
                yield ("pass", 7, step, it)
                idx += 1
                step = 1 << idx
                yield ("exchange", ["PING"], atrous_rows(step))
            yield ("pass", 10, step, it)
            fin = 2
            out_done = True
    if not out_done:
        yield ("pass", 13, fin, 0)
    yield ("pass", 14, 0, 0)


def params_dict(dp):
    """vxpt.DenoiseParams -> the switches frame_ops needs."""
    return dict(ta=bool(dp.enable_temporal_accumulation), hf=bool(dp.enable_history_fix),
                hc=bool(dp.enable_history_clamping), spatial=bool(dp.enable_spatial_filtering),
                firefly=bool(dp.enable_firefly_filter), iters=int(dp.atrous_iteration_num))


def halo_plan(bands, rank, rows):
    """{peer: ((y, n) to send, (y, n) to receive)} for the band neighbours; both
    sides of a border move min(rows, the two band heights) rows."""
    y0, y1 = bands[rank]
    plan = {}
    if rank > 0:
        n = min(rows, y1 - y0, bands[rank - 1][1] - bands[rank - 1][0])
        plan[rank - 1] = ((y0, n), (y0 - n, n))
    if rank < len(bands) - 1:
        n = min(rows, y1 - y0, bands[rank + 1][1] - bands[rank + 1][0])
        plan[rank + 1] = ((y1 - n, n), (y1, n))
    return plan


class LocalExchange:
    """Bands of one process: rows move through host memory (tests, one-GPU boxes)."""

    def __init__(self, backends, bands):
        self.backends, self.bands = backends, bands

    def __call__(self, names, rows):
        for name in names:
            full = [b.read_full(name) for b in self.backends]
            new = [f.copy() for f in full]
            for r in range(len(self.backends)):
                for peer, (_, (ry, rn)) in halo_plan(self.bands, r, rows).items():
                    new[r][ry:ry + rn] = full[peer][ry:ry + rn]
            for b, f, n in zip(self.backends, full, new):
                if not np.array_equal(f.view(np.uint8), n.view(np.uint8)):
                    b.write_full(name, n)


class DistExchange:
    """torch.distributed transport: RCCL over xGMI for GPU backends, gloo for CPU."""

    def __init__(self, backend, bands, rank, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.b, self.bands, self.rank, self.device = backend, bands, rank, device

    def __call__(self, names, rows):
        torch, dist = self.torch, self.dist
        plan = halo_plan(self.bands, self.rank, rows)
        for name in names:
            ops, recvs = [], []
            for peer, ((sy, sn), (ry, rn)) in plan.items():
                send = self.b.rows_tensor(name, sy, sn, self.device)
                recv = torch.empty_like(send) if rn == sn else self.b.rows_tensor(name, ry, rn, self.device)
                ops.append(dist.P2POp(dist.isend, send, peer))
                ops.append(dist.P2POp(dist.irecv, recv, peer))
                recvs.append((ry, rn, recv))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
                if self.device is not None:
                    torch.cuda.synchronize(self.device)
                for ry, rn, recv in recvs:
                    self.b.put_rows(name, ry, rn, recv)


def run_frame(backends, exchange, frame, spp, p, halo=(TRACE_HALO, 2), prev_halo=(TRACE_HALO, 2)):
    """Apply one frame's operations to every band backend of this process."""
    for op in frame_ops(frame, spp, p, halo, prev_halo):
        kind = op[0]
        if kind == "exchange":
            exchange(op[1], op[2])
        else:
            for b in backends:
                if kind == "trace":
                    b.trace(op[1], op[2])
                elif kind == "post_trace":
                    b.post_trace()
                else:
                    b.dpass(op[1], op[2], op[3])


class GpuBand:
    """Band backend over a vxpt.Renderer (the C ABI's band + row-copy entry points)."""

    def __init__(self, renderer, y0, y1, params):
        self.r, self.params = renderer, params
        renderer.set_band(y0, y1)

    def trace(self, it, flags):
        self.r.trace_flags(it, flags)

    def post_trace(self):
        pass

    def dpass(self, which, arg, arg2):
        self.r.denoise_pass(which, arg, arg2, self.params)

    @staticmethod
    def _name(name):  # the library's last G-buffer slot is the next trace's previous one
        return name[5:] if name.startswith("PREV:") else name

    def read_full(self, name):
        return self.r.read(self._name(name))

    def write_full(self, name, data):
        self.r.write(self._name(name), data)

    def rows_tensor(self, name, y, n, device):
        import torch
        name = self._name(name)
        rb = self.r.row_bytes(name)
        t = torch.empty(max(1, n * rb), dtype=torch.uint8, device=device)
        if n:
            self.r.copy_rows(name, y, n, t.data_ptr(), to_buffer=False)
            self.r.sync()
        return t

    def put_rows(self, name, y, n, t):
        name = self._name(name)
        if n:
            self.r.copy_rows(name, y, n, t.data_ptr(), to_buffer=True)
            self.r.sync()
