#!/bin/bash
# One band of the 8-band 1080p partition (rows 416-528) through a one-rank communicator under
# bench.band_tuning's schedule (chain gate off): kernel trace, the last frames' timeline.
# Usage (on the box): tools/kt_band_r06.sh TAG
TAG=${1:-r06band}
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="--tune state_sets=3 --tune front_streams=3 --tune iter_cap2=8 --tune resume_split=16 --tune chain_gate=0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_kt -o run -- python tools/band_kt.py 416 528 --rccl $T > gpurun_out/${TAG}_kt.log 2>&1 || { echo "band failed"; exit 1; }
python tools/timeline.py gpurun_out/${TAG}_kt/run_results.db 160 > gpurun_out/${TAG}_timeline.txt
python tools/profsum.py gpurun_out/${TAG}_kt/run_results.db 160 > gpurun_out/${TAG}_stats.txt
echo done
