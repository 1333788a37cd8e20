#!/bin/bash
# One 136-row band (rows 408-544 of the 1080p C3 frame) under bench.band_tuning's schedule: kernel
# trace, the last frame's timeline and the busy fraction.  Usage (on the box): tools/kt_band_now.sh TAG
TAG=${1:-band}
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="--tune state_sets=3 --tune front_streams=3 --tune iter_cap2=8 --tune resume_split=16"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_kt -o run -- python tools/band_kt.py 408 544 $T > gpurun_out/${TAG}_kt.log 2>&1 || { echo "band failed"; exit 1; }
python tools/timeline.py gpurun_out/${TAG}_kt/run_results.db 120 > gpurun_out/${TAG}_timeline.txt
python tools/profsum.py gpurun_out/${TAG}_kt/run_results.db 120 > gpurun_out/${TAG}_stats.txt
echo done
