#!/bin/bash
# The trace's roofline (tools/trace_roofline.py): lane DDA steps per frame from the instrumented build,
# then the product build's traversal kernels under a kernel trace and one VALU counter pass, all on the
# same 8 C3 frames with kernels one at a time.  Usage (on the box): tools/gpu_trace_roofline.sh TAG
TAG=${1:-trace}
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VXPT_LIB="$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt_stats.so" timeout -k 10 150 \
    python tools/trace_roofline.py steps gpurun_out/${TAG}_trace_steps.json > gpurun_out/${TAG}_steps.log 2>&1 || { echo "steps failed"; exit 1; }
echo steps ok
timeout -k 10 150 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_trkt -o run -- python tools/trace_roofline.py render > gpurun_out/${TAG}_trkt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
echo kt ok
timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -f csv rocpd -d gpurun_out/${TAG}_trvalu -o run -- python tools/trace_roofline.py render > gpurun_out/${TAG}_trvalu.log 2>&1 || { echo "valu pass failed"; exit 1; }
echo valu ok
python tools/trace_roofline.py combine gpurun_out/${TAG}_trace_steps.json gpurun_out/${TAG}_trvalu/run_results.db gpurun_out/${TAG}_trkt/run_results.db gpurun_out/${TAG}_trace_roofline.json
