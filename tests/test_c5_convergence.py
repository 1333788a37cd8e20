"""C5 (the canonical-render gate) at the reference's CPU frame size: 64 frames x 1 spp
of the C1 scene at 256x256, the HIP path against the oracle.  The canonical PNG the reference's
--test-canonical compares with is not shipped, so the gate is the oracle's 64-frame render, with
the bars of test_gpu_frames_spp.run_c5 (the 1920x1080 run of the same gate): relative RMS over
non-sky pixels < 1e-3 (output) / < 1e-5 (radiance), no more divergence than the reference
algorithm's own under a 1e-6 input perturbation, every pixel at or above 1e-3 listed with a cause."""
import pytest

from test_gpu_frames_spp import run_c5


@pytest.mark.gpu
def test_c5_64_frames_match_oracle():
    run_c5(256, 256, 64)
