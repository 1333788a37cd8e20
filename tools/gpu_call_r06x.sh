#!/bin/bash
# Round 6: the three-level walk ladder -- a last C3 sweep around iter_cap 4 / 6 / 12, then bands of the
# 2-, 4- and 8-band 1080p partitions with the band schedule (bench.band_tuning) against the ladder.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/tune_sweep.sh "c4a612:iter_cap=4,iter_cap2=6,iter_cap3=12" "c3a612:iter_cap=3,iter_cap2=6,iter_cap3=12" \
  "c4a512:iter_cap=4,iter_cap2=5,iter_cap3=12" "c4a610:iter_cap=4,iter_cap2=6,iter_cap3=10" \
  "c4a812:iter_cap=4,iter_cap2=8,iter_cap3=12" "c4a714:iter_cap=4,iter_cap2=7,iter_cap3=14" > gpurun_out/r06x_sweep.txt 2>&1 || exit $?
cat gpurun_out/r06x_sweep.txt
out=gpurun_out/r06x_band.txt; : > $out
for spec in "0 400 2" "400 1080 2" "200 408 4" "632 1080 4" "416 536 8"; do
  set -- $spec
  for i in 1 2; do
    for tn in "" "iter_cap=4 iter_cap2=6 iter_cap3=12"; do
      timeout -k 10 120 python -u tools/band_one.py $1 $2 $3 $tn >> $out 2>> gpurun_out/r06x_band.err || exit $?
    done
  done
done
grep '^{' $out
