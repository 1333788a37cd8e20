#!/bin/bash
# Fast GPU iteration: parity tests, short bench (no CPU baseline), kernel-trace stats.
# Usage: tools/gpu_quick.sh TAG [bench args].  Each GPU step has its own time limit.
TAG=${1:-q}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tq_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tq_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 4 --no-cpu-baseline "$@" > gpurun_out/bq_$TAG.log 2>&1 || { echo "bench failed"; tail gpurun_out/bq_$TAG.log; exit 1; }
tail -1 gpurun_out/bq_$TAG.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/pq_$TAG -o run -- python bench.py --steps 3 --warmup 8 --no-cpu-baseline "$@" > gpurun_out/pq_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
python tools/profsum.py gpurun_out/pq_$TAG/run_results.db 24
