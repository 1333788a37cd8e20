#!/bin/bash
# Round 6: the last straggler level in 32 / 64 pieces against 16 (bit-exactness, then four interleaved rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "tuning" > gpurun_out/r06ak_tests.log 2>&1 || { tail -30 gpurun_out/r06ak_tests.log; exit 1; }
tail -1 gpurun_out/r06ak_tests.log
for r in 1 2; do
bash tools/tune_sweep.sh "sp16:resume_split=16" "sp32:resume_split=32" "sp64:resume_split=64" > gpurun_out/r06ak_sweep_$r.txt 2>&1 || exit $?
cat gpurun_out/r06ak_sweep_$r.txt
done
