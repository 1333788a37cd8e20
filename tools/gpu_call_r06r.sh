#!/bin/bash
# Round 6: XCD-local work order (tuning xcd_order: k_restir / k_closest panels, k_queue runs): bit-exactness, then the C3 A/B
# (kernels alone under a kernel trace, then the pipelined bench, interleaved twice).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "xcd_order or tuning_changes_no_result" > gpurun_out/r06r_tests.log 2>&1 || { tail -30 gpurun_out/r06r_tests.log; exit 1; }
tail -2 gpurun_out/r06r_tests.log
bash tools/ab_multi.sh r06r "$L" "$L@xcd_order=1" "$L@xcd_order=2" "$L@xcd_order=4" "$L@xcd_order=7"
