#!/bin/bash
# Round 6: schedule knobs re-swept on the 4 / 6 / 12 walk ladder (tools/tune_sweep.sh, two rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/tune_sweep.sh "base:overlap=1" "wg8:resume_wg_per_cu=8" "wg24:resume_wg_per_cu=24" "wg32:resume_wg_per_cu=32" \
  "bs2:brick_steps=2" "bs4:brick_steps=4" "sp8:resume_split=8" "fs3:front_streams=3" "cam8:cam_steps=8" \
  > gpurun_out/r06aa_sweep.txt 2>&1
rc=$?; cat gpurun_out/r06aa_sweep.txt; exit $rc
