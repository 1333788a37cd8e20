"""The trace's roofline: DDA steps per second against the VALU-issue-bound peak.

The traversal kernels (k_closest: camera walks; k_queue: the queued BRDF-candidate and visibility
walks; k_resume / k_resume_split: their stragglers) are bound by instruction issue and divergence,
not by bytes.  Their roofline:
  S = lane DDA steps per frame: outer iterations (an empty-box skip or a brick entered) plus in-brick
      cell crossings, of every walk, counted by the instrumented build (libvxpt_stats.so: the same
      walks, bit for bit, with counters);
  I = the traversal kernels' SQ_INSTS_VALU per frame (wave instructions, product build);
  T = their summed kernel durations per frame (kernel trace, product build, --tune overlap=0: one
      kernel at a time);
  instructions per step = I / S; issue-bound peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU
  instruction / (I / S) lane steps per second; achieved = S / T; frac = achieved / peak (= the
  kernels' VALU issue utilisation).  With their lane utilisation u (SQ_THREAD_CYCLES_VALU / (64 x
  SQ_ACTIVE_INST_VALU)) the converged peak -- every issued instruction on 64 live lanes -- is
  peak / u, and frac_converged = frac x u.

Usage (GPU box; every run renders the same 8 C3 frames with vxpt_render_frames, --tune overlap=0):
  VXPT_LIB=.../libvxpt_stats.so python tools/trace_roofline.py steps OUT_steps.json
  rocprofv3 --kernel-trace ... -- python tools/trace_roofline.py render
  rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU ... -- python tools/trace_roofline.py render
  python tools/trace_roofline.py combine STEPS.json VALU_DB KT_DB OUT.json
"""
import collections
import ctypes
import json
import os
import re
import sqlite3
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
sys.path.insert(0, REPO)

FRAMES, SPP = 8, 4
CLOCK_HZ, SIMDS, CYCLES_PER_WAVE_OP = 2.4e9, 1024, 2
# g_stats kinds (trace.hip): 2 camera (k_closest), 1 BRDF candidates, 3 ReSTIR visibility, 4 RIS
# visibility (k_queue), 5 stragglers (k_resume), 6 straggler pieces (k_resume_split); 0 = later segments
KINDS = {0: "later-segment rays", 1: "BRDF candidates", 2: "camera", 3: "ReSTIR visibility x4",
         4: "RIS visibility", 5: "stragglers (k_resume)", 6: "straggler pieces (k_resume_split)"}
TRAVERSAL = ("k_closest", "k_queue", "k_resume", "k_resume_split")


def renderer():
    import vxpt
    from bench import C1_DIR, scene_args

    class A:
        world, scene = 256, "c3"
    chunks, hs, fd, gy, pos = scene_args(A)
    r = vxpt.Renderer(1920, 1080, device=0)
    r.load_settings()
    r.set_tuning(overlap=0)
    r.generate_terrain(chunks, height_scale=hs, freq_den=fd, global_y=gy)
    r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
    r.set_sky()
    return r, vxpt


def render():
    r, vxpt = renderer()
    r.render_frames(0, FRAMES, SPP, vxpt.DenoiseParams.defaults())
    r.sync()
    return r, vxpt


def steps(out):
    import numpy as np
    r, vxpt = renderer()
    lib = vxpt.load_library()
    lib.vxpt_debug_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(192, np.uint64)
    lib.vxpt_debug_stats(buf.ctypes.data, 1)  # reset
    r.render_frames(0, FRAMES, SPP, vxpt.DenoiseParams.defaults())
    r.sync()
    lib.vxpt_debug_stats(buf.ctypes.data, 0)
    r.close()
    kinds = {}
    for k, name in KINDS.items():
        g = [int(v) for v in buf[8 * k:8 * k + 8]]
        if g[1] == 0:
            continue
        outer = sum(g[3:7])
        kinds[name] = {"rays": g[0] / FRAMES, "waves": g[1] / FRAMES, "outer_iterations": outer / FRAMES,
                       "box_skips": sum(g[3:6]) / FRAMES, "bricks_entered": g[6] / FRAMES,
                       "cell_steps": g[7] / FRAMES, "steps": (outer + g[7]) / FRAMES,
                       "simd_eff_iterations": outer / (64.0 * g[2]) if g[2] else None}
    res = {"what": "lane DDA steps per C3 frame (1920x1080, 4 spp, 256^3 world), libvxpt_stats.so, mean of %d "
                   "frames" % FRAMES, "frames": FRAMES, "paths_per_frame": 1920 * 1080 * SPP, "kinds": kinds,
           "steps_per_frame": sum(v["steps"] for v in kinds.values())}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


def kernel_group(name):
    n = name.replace("vx::(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
    m = re.match(r"(k_[a-z_]+)", n)
    return m.group(1) if m else n


def combine(steps_json, valu_db, kt_db, out):
    st = json.load(open(steps_json))
    ins, act, thr = collections.Counter(), collections.Counter(), collections.Counter()
    for kn, cn, v in sqlite3.connect(valu_db).cursor().execute(
            "select kernel_name, counter_name, value from counters_collection"):
        g = kernel_group(kn)
        if g not in TRAVERSAL:
            continue
        {"SQ_INSTS_VALU": ins, "SQ_ACTIVE_INST_VALU": act, "SQ_THREAD_CYCLES_VALU": thr}.get(cn, collections.Counter())[g] += v
    dur, ndisp = collections.Counter(), collections.Counter()
    for n, d in sqlite3.connect(kt_db).cursor().execute("select name, duration from kernels"):
        g = kernel_group(n)
        if g in TRAVERSAL:
            dur[g] += d
            ndisp[g] += 1
    S = st["steps_per_frame"]
    I = sum(ins.values()) / FRAMES
    T = sum(dur.values()) * 1e-9 / FRAMES
    u = (sum(thr.values()) / (64.0 * sum(act.values()))) if sum(act.values()) else None
    ips = I / S
    peak = CLOCK_HZ * SIMDS / CYCLES_PER_WAVE_OP / ips
    ach = S / T
    paths = st["paths_per_frame"]
    kinds = st["kinds"]
    res = {"bound": "valu-issue", "unit": "Gsteps/s", "achieved": round(ach / 1e9, 2), "peak": round(peak / 1e9, 2),
           "frac": round(ach / peak, 4),
           "lane_util": round(u, 4) if u else None,
           "peak_converged": round(peak / u / 1e9, 2) if u else None,
           "frac_converged": round(ach / peak * u, 4) if u else None,
           "steps_per_frame": round(S), "insts_per_step": round(ips, 3),
           "traversal_ms_per_frame": round(T * 1e3, 4),
           "per_path": {"steps": round(S / paths, 2),
                        "cell_steps": round(sum(v["cell_steps"] for v in kinds.values()) / paths, 2),
                        "bricks_entered": round(sum(v["bricks_entered"] for v in kinds.values()) / paths, 2),
                        "box_skips": round(sum(v["box_skips"] for v in kinds.values()) / paths, 2),
                        "walks": round(sum(v["rays"] for k, v in kinds.items() if "pieces" not in k and "stragglers" not in k)
                                       / paths, 3)},
           "kernels": {g: {"ms_per_frame": round(dur[g] * 1e-6 / FRAMES, 4), "dispatches_per_frame": ndisp[g] / FRAMES,
                           "valu_insts_per_frame": round(ins[g] / FRAMES),
                           "lane_util": round(thr[g] / (64.0 * act[g]), 4) if act[g] else None} for g in TRAVERSAL},
           "steps_source": os.path.basename(steps_json),
           "mode": {"scene": "c3", "world": 256, "width": 1920, "height": 1080, "spp": SPP, "bounces": "3/1",
                    "primary_only": False, "tune": {"overlap": 0}, "frames": FRAMES},
           "note": "steps: libvxpt_stats.so (same walks as the product build); I, T, u: the product build, "
                   "kernels one at a time; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU op / (I / S); "
                   "frac = achieved / peak = the traversal kernels' VALU issue utilisation; frac_converged = frac x "
                   "lane utilisation (every issued op on 64 live lanes = 1)"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "steps":
        steps(sys.argv[2])
    elif cmd == "render":
        r, _ = render()
        r.close()
    elif cmd == "combine":
        combine(*sys.argv[2:6])
    else:
        raise SystemExit(__doc__)
