#!/bin/bash
# VALU issue + lane utilisation of the trace kernels: one --pmc pass (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
# SQ_THREAD_CYCLES_VALU) and a kernel-trace pass of the bench, then tools/valu_util.py.
# Usage (on the box): tools/gpu_valu.sh TAG [bench args]   -> gpurun_out/TAG_valu_util.json
TAG=${1:-valu}; shift
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS="--warmup 8 --steps 4 --no-cpu-baseline $*"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_vkt -o run -- python bench.py $ARGS > gpurun_out/${TAG}_vkt.log 2>&1 || { echo "kernel-trace pass failed"; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -f csv rocpd -d gpurun_out/${TAG}_valu -o run -- python bench.py $ARGS > gpurun_out/${TAG}_valu.log 2>&1 || { echo "valu pass failed"; exit 1; }
python tools/valu_util.py gpurun_out/${TAG}_valu/run_results.db gpurun_out/${TAG}_vkt/run_results.db gpurun_out/${TAG}_valu_util.json
