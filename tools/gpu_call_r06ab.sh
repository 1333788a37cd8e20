#!/bin/bash
# Round 6: front streams 3 and resume workgroups 24 on the walk ladder, four interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
bash tools/tune_sweep.sh "base:overlap=1" "fs3:front_streams=3" "wg24:resume_wg_per_cu=24" "fs3wg24:front_streams=3,resume_wg_per_cu=24" \
  > gpurun_out/r06ab_sweep_$r.txt 2>&1 || exit $?
cat gpurun_out/r06ab_sweep_$r.txt
done
