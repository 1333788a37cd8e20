#!/bin/bash
# round-6 call: the tuning tests (sky exit bit for bit), then the whole-frame A/B of the sky exit and one
# band's.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_dda_boxes.py tests/test_edits.py -k "tuning or probe or edit" > gpurun_out/r06k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
L="$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt.so"
bash tools/ab_multi.sh r06k5 "$L" "$L@sky_exit=0"
bash tools/gpu_call_ab_band.sh k5 libvxpt.so libvxpt.so@sky_exit=0
