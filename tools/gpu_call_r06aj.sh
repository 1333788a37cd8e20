#!/bin/bash
# Round 6: a finer direction sort (sort_mode 3: 48 classes) against sort_mode 2, four interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "tuning" > gpurun_out/r06aj_tests.log 2>&1 || { tail -30 gpurun_out/r06aj_tests.log; exit 1; }
tail -1 gpurun_out/r06aj_tests.log
for r in 1 2; do
bash tools/tune_sweep.sh "s2:sort_mode=2" "s3:sort_mode=3" > gpurun_out/r06aj_sweep_$r.txt 2>&1 || exit $?
cat gpurun_out/r06aj_sweep_$r.txt
done
