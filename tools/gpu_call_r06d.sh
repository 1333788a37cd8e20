#!/bin/bash
# round-6 call: band proxy with the banded schedule (chain_gate 0), the tests of the band / tuning code,
# then an A/B of the whole-frame loop (chain gate off; the temporal pass at 5 waves).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/band_proxy.py --out gpurun_out/r06b_band_proxy.json > gpurun_out/r06b_band_proxy.log 2>&1 || exit $?
echo proxy ok
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bands.py tests/test_gpu_parity.py -k "band or tuning or linked or rccl" > gpurun_out/r06d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
bash tools/ab_multi.sh r06d "$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt.so" "$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt.so@chain_gate=0" "$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt_ta5.so"
