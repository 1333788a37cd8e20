"""Band backend over the oracle (test infrastructure): lets the multi-GPU band
schedule of bands.py run on CPU, in one process or over gloo."""
import numpy as np

IDS = dict(ILLUM=0, DEPTH=1, NORMAL_ROUGH=2, GEO_NORMAL_THIN=3, ALBEDO=4, MATERIAL=5, MAT_PARAM=6, PING=15,
           PONG=16, PREV_ILLUM=17, PREV_FAST=18, HIST_LEN=19, PREV_HIST_LEN=20, OUTPUT=21)
# the previous pass's G-buffer the oracle's next trace reads: its Prev* copies
IDS.update({"PREV:NORMAL_ROUGH": 8, "PREV:GEO_NORMAL_THIN": 9, "PREV:ALBEDO": 10, "PREV:MAT_PARAM": 11,
            "PREV:DEPTH": 12, "PREV:MATERIAL": 13})
COPY_SRC = {0: 0, 1: 15, 2: 16, 3: 17}


class OracleBand:
    def __init__(self, o, y0, y1):
        self.o, self.y0, self.y1 = o, y0, y1
        o.set_band(y0, y1)

    def trace(self, it, flags):
        assert flags == 0, "the oracle restates spp = 1 passes"
        self.o.trace(it, self.y0, self.y1)

    def post_trace(self):
        self.o.post_trace()

    def dpass(self, which, arg, arg2):
        o = self.o
        if which in (0, 2, 3, 4, 5):
            o.run_pass(which, arg, arg2)
        elif which in (6, 7):
            o.run_pass(which, arg, arg2)
        elif which == 10:  # final a-trous + output (sky copy + remodulated non-sky)
            o.run_pass(6, arg, arg2)
            o.run_pass(1)
            o.run_pass(8, 16)
        elif which == 12:
            o.run_pass(10)
        elif which == 13:
            o.run_pass(1)
            o.run_pass(8, COPY_SRC[arg])
        elif which == 14:
            o.run_pass(9)
        elif which != 11:  # 11: world positions are computed inline by the oracle
            raise ValueError(which)

    def read_full(self, name):
        if name.startswith("RES_"):
            par = 0 if name == "RES_EVEN" else 1
            n = self.o.W * self.o.H
            return self.o.read(14)[par * n:(par + 1) * n].reshape(self.o.H, self.o.W).copy()
        return self.o.read(IDS[name])

    def write_full(self, name, data):
        if name.startswith("RES_"):
            par = 0 if name == "RES_EVEN" else 1
            n = self.o.W * self.o.H
            full = self.o.read(14)
            full[par * n:(par + 1) * n] = np.ascontiguousarray(data).reshape(-1)
            self.o.write(14, full)
        else:
            self.o.write(IDS[name], data)

    def rows_tensor(self, name, y, n, device=None):
        import torch
        rows = np.ascontiguousarray(self.read_full(name)[y:y + n])
        return torch.from_numpy(rows.view(np.uint8).reshape(-1).copy())

    def put_rows(self, name, y, n, t):
        arr = self.read_full(name)
        arr[y:y + n] = t.numpy().view(arr.dtype).reshape(arr[y:y + n].shape)
        self.write_full(name, arr)
