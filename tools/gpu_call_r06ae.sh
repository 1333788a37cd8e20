#!/bin/bash
# Round 6: direction sort with larger box growth limits, four interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
bash tools/tune_sweep.sh "s1bc32:sort_mode=1,box_cap=32,box_cap_up=32" "s2bc32:sort_mode=2,box_cap=32,box_cap_up=32" \
  "s1bc64:sort_mode=1,box_cap=64,box_cap_up=64" "s2bc64:sort_mode=2,box_cap=64,box_cap_up=64" \
  "s1bc32u64:sort_mode=1,box_cap=32,box_cap_up=64" "s1bc128:sort_mode=1,box_cap=128,box_cap_up=128" \
  "s1bc64u32:sort_mode=1,box_cap=64,box_cap_up=32" > gpurun_out/r06ae_sweep_$r.txt 2>&1 || exit $?
cat gpurun_out/r06ae_sweep_$r.txt
done
