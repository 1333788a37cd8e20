#!/bin/bash
# A/B of the first-half stream / state-set settings: the tuning tests, the C3 bench (two rounds) and
# one 8-band rank (rows 408-544) and an 8-row band.  Usage (on the box): tools/fs_ab.sh "NAME:field=v,..." ...
export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "tuning or pipelined or overlapped" > gpurun_out/fs_tests.log 2>&1; echo trc=$?; tail -2 gpurun_out/fs_tests.log
bash tools/tune_sweep.sh "$@" || exit 1
for spec in "$@"; do
  vals=${spec#*:}; args=""
  for kv in ${vals//,/ }; do args="$args --tune $kv"; done
  echo "${spec%%:*}"
  timeout -k 10 100 python tools/band_kt.py 408 544 $args || exit 1
  timeout -k 10 100 python tools/band_kt.py 408 416 $args || exit 1
done
