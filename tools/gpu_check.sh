#!/bin/bash
# GPU-box routine: parity tests, bench, kernel-trace profile.  Usage: tools/gpu_check.sh TAG [bench args]
# Each GPU step has its own time limit; a failing step ends the script.
TAG=${1:-run}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rA > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed rc=$?"; exit 1; }
echo bench ok
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 4 --warmup 4 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "prof rc=$?"
