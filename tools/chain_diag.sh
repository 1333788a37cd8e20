#!/bin/bash
# Why a pipelined frame's denoiser chain runs slower than a frame-by-frame one: per chain kernel, the
# kernel-trace duration, the shader clock (GRBM_GUI_ACTIVE cycles / duration) and the UTCL1
# translation miss rate, for both frame loops.  Usage (on the box): tools/chain_diag.sh TAG
TAG=${1:-cd}
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mode in pipe calls; do
    extra=""
    [ $mode = calls ] && extra="--frame-calls"
    ARGS="--warmup 8 --steps 6 --no-cpu-baseline $extra"
    timeout -k 10 200 rocprofv3 --kernel-trace -f csv rocpd -d gpurun_out/${TAG}_${mode}_kt -o run -- python bench.py $ARGS > gpurun_out/${TAG}_${mode}_kt.log 2>&1 || { echo "kt $mode failed"; exit 1; }
    timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum -f csv rocpd -d gpurun_out/${TAG}_${mode}_pmc -o run -- python bench.py $ARGS > gpurun_out/${TAG}_${mode}_pmc.log 2>&1 || { echo "pmc $mode failed"; exit 1; }
done
python tools/chain_diag.py gpurun_out/${TAG} > gpurun_out/${TAG}_chain_diag.txt
