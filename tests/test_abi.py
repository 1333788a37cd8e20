"""CPU tests of the drop-in boundary: libvxpt.so (HIP for gfx950 + C++ host)
loads, exports every entry point include/vxpt.h declares, carries gfx950 code
objects, and refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "vxpt.h")
LIB = os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd", "libvxpt.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vxpt_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("vxpt_create", "vxpt_destroy", "vxpt_trace", "vxpt_denoise", "vxpt_render_frame",
                 "vxpt_set_sky", "vxpt_readback", "vxpt_probe_rays"):
        assert must in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "libvxpt.so not built: run __graft_entry__.build()"
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_has_gfx950_code_object():
    # the fat binary embeds the offload bundle id of every device code object
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_python_mirror_binds_all_symbols():
    import vxpt
    lib = vxpt.load_library()
    for n in declared():
        assert hasattr(lib, n)


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import vxpt
    with pytest.raises(vxpt.VxptError):
        vxpt.Renderer(64, 64)
