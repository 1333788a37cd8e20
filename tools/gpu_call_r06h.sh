#!/bin/bash
# round-6 call: the tuning / band tests with four state sets, then the band A/B of state sets.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bands.py tests/test_gpu_parity.py -k "tuning or linked_render_frames or library_band" > gpurun_out/r06h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_call_ab_band.sh h1 libvxpt.so libvxpt.so@state_sets=4 libvxpt.so@state_sets=4@front_streams=4
