#!/bin/bash
# Round 6: the remaining schedule knobs on the final tree (tools/tune_sweep.sh, two rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/tune_sweep.sh "base:overlap=1" "sort1:sort_mode=1" "sort2:sort_mode=2" "rw4:restir_waves=4" \
  "ss2:state_sets=2" "fs3:front_streams=3" "bc16:box_cap=16,box_cap_up=16" > gpurun_out/r06ac_sweep.txt 2>&1
rc=$?; cat gpurun_out/r06ac_sweep.txt; exit $rc
