#!/bin/bash
# Kernel-trace profile of the bench workload, plus the traversal statistics build.
# Usage (on the box): tools/gpu_kt.sh TAG [bench args]   -> gpurun_out/TAG_kt.txt, gpurun_out/TAG_stats.txt
# Bench args (e.g. --tune overlap=0) pass through to the kernel trace.
TAG=${1:-kt}; shift
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_kt -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline "$@" > gpurun_out/${TAG}_kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
python tools/profsum.py gpurun_out/${TAG}_kt/run_results.db 40 > gpurun_out/${TAG}_kt.txt
if [ -f real-time-path-tracing-voxel-blocks_amd/libvxpt_stats.so ]; then
    VXPT_LIB=real-time-path-tracing-voxel-blocks_amd/libvxpt_stats.so timeout -k 10 200 python tools/trace_stats.py > gpurun_out/${TAG}_stats.txt 2>&1 || { echo "stats failed"; exit 1; }
fi
echo "$TAG done"
