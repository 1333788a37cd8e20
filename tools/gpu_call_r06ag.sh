#!/bin/bash
# Round 6: the walk ladder and walk knobs re-swept with the sort and 32-brick boxes (tune_sweep, two rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/tune_sweep.sh "base:overlap=1" "c5:iter_cap=5" "c3:iter_cap=3" "a512:iter_cap2=5,iter_cap3=12" \
  "a616:iter_cap2=6,iter_cap3=16" "a79:iter_cap2=7,iter_cap3=9" "bs4:brick_steps=4" "cam12:cam_steps=12" \
  "fs3:front_streams=3" "wg32:resume_wg_per_cu=32" "sp8:resume_split=8" > gpurun_out/r06ag_sweep.txt 2>&1
rc=$?; cat gpurun_out/r06ag_sweep.txt; exit $rc
