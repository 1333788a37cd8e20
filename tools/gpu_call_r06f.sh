#!/bin/bash
# round-6 call: the turning-camera band tests (ghost rows with a history halo deeper than their margin),
# then the 4K band proxy (BASELINE config 3's size) with the round-6 band schedule.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bands.py -k "turning or translating" > gpurun_out/r06f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 800 python -u tools/band_proxy.py 3840 2160 --out gpurun_out/r06b_band_proxy_4k.json > gpurun_out/r06b_band_proxy_4k.log 2>&1 || exit $?
echo proxy ok
