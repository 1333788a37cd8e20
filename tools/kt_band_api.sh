#!/bin/bash
# One band of the 8-band 1080p partition through a one-rank communicator under bench.band_tuning's
# schedule, with the HIP API trace beside the kernel trace: where the host blocks while it enqueues a
# banded frame.  Usage (on the box): tools/kt_band_api.sh TAG
TAG=${1:-r06api}
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="--tune state_sets=3 --tune front_streams=3 --tune iter_cap2=8 --tune resume_split=16 --tune chain_gate=0"
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG} -o run -- python tools/band_kt.py 416 528 --rccl --frames 4 --warmup 4 $T > gpurun_out/${TAG}.log 2>&1 || { echo "band failed"; exit 1; }
python tools/timeline.py gpurun_out/${TAG}/run_results.db 160 > gpurun_out/${TAG}_timeline.txt
echo done
