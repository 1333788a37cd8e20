#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, no trace domains) + kernel trace,
# steady-state frames, and the FETCH_SIZE / WRITE_SIZE calibration per access width.
# Usage: tools/gpu_pmc.sh TAG [bench args]   -> gpurun_out/TAG_*.{db,json,txt}
TAG=${1:-pmc}; shift
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS="--warmup 8 --steps 4 --no-cpu-baseline $*"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -f csv rocpd -d gpurun_out/${TAG}_cfetch -o run -- ./tools/calib/pmc_calib > gpurun_out/${TAG}_cfetch.log 2>&1 || { echo "calib fetch failed"; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -f csv rocpd -d gpurun_out/${TAG}_cwrite -o run -- ./tools/calib/pmc_calib > gpurun_out/${TAG}_cwrite.log 2>&1 || { echo "calib write failed"; exit 1; }
python tools/pmc_calib.py gpurun_out/${TAG}_cfetch/run_results.db gpurun_out/${TAG}_cwrite/run_results.db gpurun_out/${TAG}_pmc_calib.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_kt -o run -- python bench.py $ARGS > gpurun_out/${TAG}_kt.log 2>&1 || { echo "kernel-trace pass failed"; exit 1; }
echo kt ok
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -f csv rocpd -d gpurun_out/${TAG}_fetch -o run -- python bench.py $ARGS > gpurun_out/${TAG}_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo fetch ok
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -f csv rocpd -d gpurun_out/${TAG}_write -o run -- python bench.py $ARGS > gpurun_out/${TAG}_write.log 2>&1 || { echo "write pass failed"; exit 1; }
echo write ok
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES -f csv rocpd -d gpurun_out/${TAG}_sq -o run -- python bench.py $ARGS > gpurun_out/${TAG}_sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
echo sq ok
python tools/pmc_traffic.py gpurun_out/${TAG}_fetch/run_results.db gpurun_out/${TAG}_write/run_results.db gpurun_out/${TAG}_kt/run_results.db 4 gpurun_out/${TAG}_pmc_denoise.json gpurun_out/${TAG}_pmc_calib.json gpurun_out/${TAG}_kt.log
python tools/pmcsum.py gpurun_out/${TAG}_sq/run_results.db gpurun_out/${TAG}_fetch/run_results.db gpurun_out/${TAG}_write/run_results.db > gpurun_out/${TAG}_pmc.txt
python tools/profsum.py gpurun_out/${TAG}_kt/run_results.db > gpurun_out/${TAG}_kernel_stats.txt
# VALU lane activity (divergence) when the device exposes the counters (rocprofv3 -L); the issue
# utilisation needs only the SQ pass above
if grep -q "SQ_THREAD_CYCLES_VALU" gpurun_out/counters.txt 2>/dev/null && grep -q "SQ_ACTIVE_INST_VALU" gpurun_out/counters.txt; then
    timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -f csv rocpd -d gpurun_out/${TAG}_valu -o run -- python bench.py $ARGS > gpurun_out/${TAG}_valu.log 2>&1 || { echo "valu pass failed"; exit 1; }
    python tools/valu_util.py gpurun_out/${TAG}_valu/run_results.db gpurun_out/${TAG}_kt/run_results.db gpurun_out/${TAG}_valu_util.json gpurun_out/${TAG}_kt.log
else
    python tools/valu_util.py gpurun_out/${TAG}_sq/run_results.db gpurun_out/${TAG}_kt/run_results.db gpurun_out/${TAG}_valu_util.json gpurun_out/${TAG}_kt.log
fi
