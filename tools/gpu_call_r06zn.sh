#!/bin/bash
# Round 6, the final tree (walk ladder, 24 resume workgroups per CU, sort 2, 32-brick boxes): every GPU test, the bench lines, the PMC / VALU
# passes and the trace roofline (tag r06zn), then the band proxy with bench.band_tuning's schedules.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_batch.sh counters || exit $?
bash tools/gpu_batch.sh tests
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_batch.sh full c2 b44 bands1 || exit $?
bash tools/gpu_pmc.sh r06zn > gpurun_out/r06zn_pmc_run.log 2>&1; echo "pmc rc=$?"
bash tools/gpu_trace_roofline.sh r06zn; echo "trace roofline rc=$?"
timeout -k 10 400 python -u tools/band_proxy.py --out gpurun_out/r06g_band_proxy.json > gpurun_out/r06g_band_proxy.log 2>&1; echo "proxy rc=$?"
timeout -k 10 600 python -u tools/band_proxy.py 3840 2160 --out gpurun_out/r06g_band_proxy_4k.json > gpurun_out/r06g_band_proxy_4k.log 2>&1; echo "proxy 4k rc=$?"
