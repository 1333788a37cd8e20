"""The offline renderer executable (csrc/vxpt_offline.cpp), the reference's
mainOffline.cpp over the C ABI: its flags, its output files (<prefix>_%04d.png
for the 1-indexed frames {1, 4, 16, 64}, named by the 0-indexed frame) and the
canonical-image gate (mainOffline.cpp:423-498).

CPU: argument handling (help, bad sizes, the unsupported scripted-edit flags).
GPU: a short run writes the reference's file set, the canonical gate reports
IDENTICAL against its own update, and the saved frame is bit-identical to the
same frames rendered through the Python mirror of the same entry points.
"""
import os
import subprocess

import numpy as np
import pytest

import vxpt

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd", "vxpt_offline")


def run(*args, timeout=60):
    return subprocess.run([EXE, *args], cwd=REPO, capture_output=True, text=True, timeout=timeout)


def test_cli_built_and_help():
    assert os.path.exists(EXE), "vxpt_offline not built: run __graft_entry__.build()"
    r = run("--help")
    assert r.returncode == 0
    for flag in ("--width", "--height", "--output", "--scene", "--test-canonical", "--update-canonical",
                 "--canonical-image", "--comment", "--frames"):
        assert flag in r.stdout


@pytest.mark.parametrize("args", [("--width", "0"), ("--frames", "0"), ("--chunks", "2", "1")])
def test_cli_rejects_bad_arguments(args):
    r = run(*args)
    assert r.returncode == 2, (r.stdout, r.stderr)


@pytest.mark.parametrize("args", [("--bogus", "--help"), ("--help", "--output"), ("--some-new-flag", "7", "--help")])
def test_cli_ignores_unknown_and_valueless_flags(args):
    """mainOffline.cpp:57-133 skips arguments it does not know and a trailing flag without
    its value; reference scripts with extra flags must run unchanged."""
    r = run(*args)
    assert r.returncode == 0, (r.stdout, r.stderr)


@pytest.mark.gpu
def test_cli_offline_run_and_canonical_gate(tmp_path):
    w, h, frames = 128, 96, 4
    prefix = str(tmp_path / "off")
    canon = str(tmp_path / "canon.png")
    r = run("--width", str(w), "--height", str(h), "--frames", str(frames), "--output", prefix,
            "--update-canonical", "--test-canonical", "--canonical-image", canon, "--comment", "cli test",
            "--perf-report", str(tmp_path / "perf" / "performance_report.txt"), timeout=120)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    # frames 1 and 4 (1-indexed) are saved under their 0-indexed numbers
    for f in (0, 3):
        assert os.path.exists("%s_%04d.png" % (prefix, f))
    assert not os.path.exists("%s_%04d.png" % (prefix, 1))
    assert "Assessment: IDENTICAL" in r.stdout and os.path.exists(prefix + "_diff.png")
    assert os.path.exists(prefix + "_frames.csv")
    # PerformanceTracker::saveReport's run summary (PerformanceTracker.h:98-183), header included
    rep = open(tmp_path / "perf" / "performance_report.txt").read().splitlines()
    assert rep[0].startswith("# Performance Report") and rep[1].startswith("# Format: Timestamp") and len(rep) == 4
    cols = [c.strip() for c in rep[3].split("|")]
    assert len(cols) == 11 and cols[1] == str(frames) and cols[2] == "%dx%d" % (w, h) and cols[10] == "cli test"
    assert float(cols[7]) > 0.0 and float(cols[8]) > 0.0  # path tracing, denoiser ms

    # the same frames through the Python mirror of the same entry points
    rr = vxpt.Renderer(w, h)
    rr.load_settings()
    rr.generate_terrain((2, 1, 2))
    cam = rr.scene_camera(os.path.join(REPO, "data", "scene", "scene_export.yaml"))
    c = (list(cam.pos), list(cam.dir), cam.fov_deg)
    rr.set_camera(*c[:2], fov=c[2], prev=c)
    rr.set_sky()
    dp, pp = rr.denoise_params(), rr.post_params()
    # the CLI's frame times (Timer::getDeltaTime) drive the exposure adaptation: replay them
    rows = [ln.split(",") for ln in open(prefix + "_frames.csv") if ln[0].isdigit()]
    dts = [float(x[7]) for x in rows]
    assert len(dts) == frames
    for f in range(frames):
        rr.render_frame(f, 1, dp)
        rr.postprocess(pp, dts[f])
    mine = str(tmp_path / "py.png")
    rr.write_png(mine)
    rr.close()
    a, b = vxpt.read_png(mine), vxpt.read_png("%s_%04d.png" % (prefix, frames - 1))
    np.testing.assert_array_equal(a, b)
    assert a.std() > 1.0  # a real image, not a blank frame
