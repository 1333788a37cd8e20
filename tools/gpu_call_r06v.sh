#!/bin/bash
# Round 6: the three-level straggler schedule swept on C3 (tools/tune_sweep.sh, two rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/tune_sweep.sh "base:overlap=1" "a88:iter_cap2=8,iter_cap3=8" "a68:iter_cap2=6,iter_cap3=8" \
  "a66:iter_cap2=6,iter_cap3=6" "a612:iter_cap2=6,iter_cap3=12" "a812:iter_cap2=8,iter_cap3=12" \
  "a86:iter_cap2=8,iter_cap3=6" "c4a88:iter_cap=4,iter_cap2=8,iter_cap3=8" "c6a88:iter_cap=6,iter_cap2=8,iter_cap3=8" \
  "s8a88:resume_split=8,iter_cap2=8,iter_cap3=8" "a55:iter_cap2=5,iter_cap3=5" > gpurun_out/r06v_sweep.txt 2>&1
rc=$?; cat gpurun_out/r06v_sweep.txt; exit $rc
