#!/bin/bash
# The round's GPU evidence in one call: rocprofv3 -L, every GPU test, the default bench line with the
# CPU baseline, the C2 primary-only and 4/4-bounce lines, and the profile passes (kernel trace, PMC,
# VALU lane utilisation) of tools/gpu_pmc.sh.
# Usage (on the box): tools/gpu_round.sh TAG
TAG=${1:-r03}
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_batch.sh counters || exit $?
bash tools/gpu_batch.sh tests
rc=$?
echo "tests rc=$rc"
# a failing assertion (pytest 1) does not stop the measurements; a crash, fault or timeout does
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_batch.sh full c2 b44 || exit $?
bash tools/gpu_pmc.sh "$TAG" > gpurun_out/${TAG}_pmc_run.log 2>&1; echo "pmc rc=$?"
