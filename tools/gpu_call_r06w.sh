#!/bin/bash
# Round 6: the multi-level straggler schedule swept further on C3 (tools/tune_sweep.sh, two rounds);
# iter_cap4 adds a fourth capped level.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "tuning_changes_no_result" > gpurun_out/r06w_tests.log 2>&1 || { tail -30 gpurun_out/r06w_tests.log; exit 1; }
tail -1 gpurun_out/r06w_tests.log
bash tools/tune_sweep.sh "base:overlap=1" "a612:iter_cap2=6,iter_cap3=12" "a616:iter_cap2=6,iter_cap3=16" \
  "a624:iter_cap2=6,iter_cap3=24" "a412:iter_cap2=4,iter_cap3=12" "a416:iter_cap2=4,iter_cap3=16" \
  "b6812:iter_cap2=6,iter_cap3=8,iter_cap4=12" "b4816:iter_cap2=4,iter_cap3=8,iter_cap4=16" \
  "b6612:iter_cap2=6,iter_cap3=6,iter_cap4=12" "s8a612:resume_split=8,iter_cap2=6,iter_cap3=12" \
  "c4a612:iter_cap=4,iter_cap2=6,iter_cap3=12" "c4s8a612:iter_cap=4,resume_split=8,iter_cap2=6,iter_cap3=12" \
  > gpurun_out/r06w_sweep.txt 2>&1
rc=$?; cat gpurun_out/r06w_sweep.txt; exit $rc
