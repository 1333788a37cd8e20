#!/bin/bash
# The band-partition proxy of this round's schedule (ghost rows on, the default) and of the per-pass
# exchange schedule (ghost_rows 0), each step under its own limit.  Usage (on the box).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 540 python -u tools/band_proxy.py --out gpurun_out/r06_band_proxy.json > gpurun_out/r06_band_proxy.log 2>&1 || exit $?
echo proxy ok
timeout -k 10 540 python -u tools/band_proxy.py --tune ghost_rows=0 --out gpurun_out/r06_band_proxy_noghost.json > gpurun_out/r06_band_proxy_noghost.log 2>&1 || exit $?
echo noghost ok
