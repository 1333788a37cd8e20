#!/bin/bash
# round-6 call: the band and tuning tests on the final defaults, then the 1080p band proxy.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_bands.py tests/test_gpu_parity.py -k "band or tuning or linked or rccl" > gpurun_out/r06o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/band_proxy.py --out gpurun_out/r06c_band_proxy.json > gpurun_out/r06c_band_proxy.log 2>&1 || exit $?
echo proxy ok
