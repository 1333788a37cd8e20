"""RCCL band schedule check on one device (GPU-box diagnostic).

Launched with torch.distributed.run --nproc-per-node 2: both ranks use device 0
(a one-GPU box), the unique id travels over gloo, and each rank renders its band
with the library's RCCL halo exchanges; rank 0 compares the gathered output with
a single-context render.  RCCL may refuse two ranks on one device -- then the
check reports that and exits 0 (the linked-context test covers the schedule).
On a multi-GPU box each rank takes device LOCAL_RANK.  --uneven: the 2-rank
partition [0, 88, 160] (vxpt_band_comm_init_rows) instead of the equal bands.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bands  # noqa: E402
import vxpt  # noqa: E402
from golden.make_golden import C1_CAMERA  # noqa: E402

W, H, SPP = 64, 160, 4
DEV = 0


def make():
    r = vxpt.Renderer(W, H, device=DEV)
    r.load_settings()
    r.generate_terrain((2, 1, 2))
    r.set_camera(*C1_CAMERA[:2], fov=C1_CAMERA[2], prev=C1_CAMERA)
    r.set_sky()
    return r


def main():
    global DEV
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import torch
    n = torch.cuda.device_count()
    DEV = int(os.environ.get("LOCAL_RANK", 0)) % max(n, 1)
    splits = [0, 88, 160] if "--uneven" in sys.argv and world == 2 else None
    obj = [vxpt.band_comm_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    r = make()
    try:
        r.band_comm_init(obj[0], world, rank, splits)
    except vxpt.VxptError as e:
        print("rank %d: RCCL refused (%s); schedule covered by the linked-context test" % (rank, e), flush=True)
        return
    p = vxpt.DenoiseParams.defaults()
    y0, y1 = bands.band_rows(H, world, rank) if splits is None else (splits[rank], splits[rank + 1])
    outs = []
    for f in range(3):
        r.render_frame(f, SPP, p)
        outs.append(r.read("OUTPUT")[y0:y1].copy())
    gathered = [None] * world
    dist.all_gather_object(gathered, outs)
    if rank == 0:
        single = make()
        for f in range(3):
            single.render_frame(f, SPP, p)
            ref = single.read("OUTPUT")
            out = np.concatenate([g[f] for g in gathered])
            same = np.array_equal(out.view(np.uint32), ref.view(np.uint32))
            print("frame %d: RCCL bands bit-exact vs single context: %s" % (f, same), flush=True)
            assert same
        print("RCCL band schedule OK; timings", r.timings(), flush=True)


if __name__ == "__main__":
    main()
