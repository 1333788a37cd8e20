#!/bin/bash
# Round 6: direction sort 2 with 32-brick box growth limits on bands of the 8- and 2-band 1080p partitions.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r06af_band.txt; : > $out
for spec in "416 536 8" "0 104 8" "832 1080 8" "0 400 2" "200 408 4"; do
  set -- $spec
  for i in 1 2; do
    for tn in "" "sort_mode=2 box_cap=32 box_cap_up=32" "box_cap=32 box_cap_up=32"; do
      timeout -k 10 120 python -u tools/band_one.py $1 $2 $3 $tn >> $out 2>> gpurun_out/r06af_band.err || exit $?
    done
  done
done
grep '^{' $out
