#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, no trace domains).
# Usage: tools/gpu_pmc.sh TAG [bench args]
TAG=${1:-pmc}; shift
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS="$@"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU -f csv rocpd -d gpurun_out/${TAG}_sq -o run -- python bench.py $ARGS > gpurun_out/${TAG}_sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
echo sq ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv rocpd -d gpurun_out/${TAG}_fetch -o run -- python bench.py $ARGS > gpurun_out/${TAG}_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv rocpd -d gpurun_out/${TAG}_write -o run -- python bench.py $ARGS > gpurun_out/${TAG}_write.log 2>&1 || { echo "write pass failed"; exit 1; }
echo write ok
