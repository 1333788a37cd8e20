#!/bin/bash
# One GPU call's worth of round-2 checks, each step under its own time limit; stops at the first
# GPU fault / timeout.  Usage (on the box): tools/gpu_batch.sh STEP...   steps:
#   tests    pytest -m gpu on the files in $TESTS (default: all)
#   bench    bench.py --steps 20 --warmup 6 --no-cpu-baseline  -> gpurun_out/b_default.json
#   full     bench.py (defaults, CPU baseline on)                          -> gpurun_out/b_full.json
#   c2       bench.py --primary-only                                       -> gpurun_out/b_c2.json
#   b44      bench.py --bounces 4/4 --no-cpu-baseline                      -> gpurun_out/b_44.json
#   bands1   bench.py --bands (the banded path over a one-rank communicator, band_parity) -> gpurun_out/b_bands1.json
#   counters rocprofv3 -L                                                  -> gpurun_out/counters.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$secs" "$@"
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for step in "$@"; do
    case $step in
    tests) run tests 900 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu ${TESTS:-tests} \
               > gpurun_out/tests.log 2>&1 || exit $? ;;
    bench) run bench 200 python -u bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/b_default.json 2> gpurun_out/b_default.err || exit $? ;;
    full) run full 400 python -u bench.py > gpurun_out/b_full.json 2> gpurun_out/b_full.err || exit $? ;;
    c2) run c2 300 python -u bench.py --primary-only --cpu-seconds 8 > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || exit $? ;;
    b44) run b44 200 python -u bench.py --bounces 4/4 --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/b_44.json 2> gpurun_out/b_44.err || exit $? ;;
    bands1) run bands1 300 python -u bench.py --bands --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/b_bands1.json 2> gpurun_out/b_bands1.err || exit $? ;;
    counters) (cd /tmp && TMPDIR=/tmp timeout -k 5 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters.txt" 2>&1); true ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
