"""Runs tools/dda_sim/tile_working_set.hip (the library's walk on the host) on the bench workload:
the C3 world (256^3, bench.py scene_args) at 1920x1080 from the bench camera.  CPU study, not
product code.  Usage: python tools/dda_sim/tile_working_set.py [W H]"""
import os
import subprocess
import sys
import tempfile

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(REPO, d) for d in ("oracle", "tests")]
import numpy as np
import oracle
from golden.make_golden import C1_CAMERA

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1080)
d = tempfile.mkdtemp()
exe = os.path.join(d, "tws")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                       "-I", os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd", "csrc"), "-x", "hip",
                       os.path.join(REPO, "tools", "dda_sim", "tile_working_set.hip"), "-o", exe])
o = oracle.Oracle(W, H)
o.terrain((8, 8, 8), height_scale=128.0, freq_den=256.0, global_y=True)
pos = [p * 4 for p in C1_CAMERA[0]]
o.set_camera(pos, C1_CAMERA[1], fov=90.0)
o.voxels().astype(np.uint8).tofile(os.path.join(d, "ids.bin"))
np.asarray(o.camera_info(0), np.float32)[:32].tofile(os.path.join(d, "cam.bin"))
print(subprocess.run([exe, os.path.join(d, "ids.bin"), "8", "8", "8", os.path.join(d, "cam.bin"), str(W), str(H)],
                     check=True, capture_output=True, text=True).stdout)
