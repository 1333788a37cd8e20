#!/bin/bash
# Round 6, final tree: rocprofv3 -L, every GPU test, the bench lines (full with the CPU baseline, C2,
# 4/4 bounces, the banded path over a one-rank communicator), then the PMC / VALU passes and the trace
# roofline.  Each step under its own time limit (tools/gpu_batch.sh, gpu_pmc.sh, gpu_trace_roofline.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_batch.sh counters || exit $?
bash tools/gpu_batch.sh tests
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_batch.sh full c2 b44 bands1 || exit $?
bash tools/gpu_pmc.sh r06z > gpurun_out/r06z_pmc_run.log 2>&1; echo "pmc rc=$?"
bash tools/gpu_trace_roofline.sh r06z; echo "trace roofline rc=$?"
