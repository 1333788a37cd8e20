#!/bin/bash
# Round 6: direction sort and box growth limits on the walk ladder, four interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
bash tools/tune_sweep.sh "base:overlap=1" "sort1:sort_mode=1" "bc16:box_cap=16,box_cap_up=16" \
  "s1bc16:sort_mode=1,box_cap=16,box_cap_up=16" "s2bc16:sort_mode=2,box_cap=16,box_cap_up=16" \
  "bc32:box_cap=32,box_cap_up=32" "s1bc32:sort_mode=1,box_cap=32,box_cap_up=32" "bc8u16:box_cap=8,box_cap_up=16" \
  > gpurun_out/r06ad_sweep_$r.txt 2>&1 || exit $?
cat gpurun_out/r06ad_sweep_$r.txt
done
