#!/bin/bash
# Round 6: a third straggler level (tuning iter_cap3): bit-exactness, the C3 A/B, then bands.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "tuning_changes_no_result" > gpurun_out/r06u_tests.log 2>&1 || { tail -30 gpurun_out/r06u_tests.log; exit 1; }
tail -2 gpurun_out/r06u_tests.log
bash tools/ab_multi.sh r06u "$L" "$L@iter_cap2=8@iter_cap3=8" "$L@iter_cap2=10@iter_cap3=12" "$L@iter_cap2=16@iter_cap3=16" || exit 1
bash tools/gpu_call_ab_band.sh r06u libvxpt.so libvxpt.so@iter_cap3=8 libvxpt.so@iter_cap2=4@iter_cap3=6
