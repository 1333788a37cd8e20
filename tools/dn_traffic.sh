#!/bin/bash
# Denoiser chain traffic (FETCH_SIZE / WRITE_SIZE passes + kernel trace) for one setting:
# tools/dn_traffic.sh TAG [VAR=VAL ...]  -> gpurun_out/TAG_pmc_denoise.json (calibration: profiles/r03_pmc_calib.json)
TAG=$1; shift
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS="--warmup 8 --steps 4 --no-cpu-baseline"
env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_kt -o run -- python bench.py $ARGS > gpurun_out/${TAG}_kt.log 2>&1 || exit 1
env "$@" timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -f csv rocpd -d gpurun_out/${TAG}_fetch -o run -- python bench.py $ARGS > gpurun_out/${TAG}_fetch.log 2>&1 || exit 1
env "$@" timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -f csv rocpd -d gpurun_out/${TAG}_write -o run -- python bench.py $ARGS > gpurun_out/${TAG}_write.log 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/${TAG}_fetch/run_results.db gpurun_out/${TAG}_write/run_results.db gpurun_out/${TAG}_kt/run_results.db 4 gpurun_out/${TAG}_pmc_denoise.json profiles/r03_pmc_calib.json
