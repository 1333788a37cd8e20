#!/bin/bash
# A/B on single 1080p bands of the 8-band partition through a one-rank communicator (tools/band_one.py),
# interleaved twice: VARIANT = LIB[@field=value...] (the fields go to band_one.py as tuning).
# Usage (on the box): tools/gpu_call_ab_band.sh TAG VARIANT...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${TAG}_ab_band.txt
: > $out
for rows in "416 536" "832 1080" "0 104"; do
  for i in 1 2; do
    for v in "$@"; do
      lib=${v%%@*}; tn=""
      [ "$lib" != "$v" ] && tn=$(echo "${v#*@}" | tr '@' ' ')
      VXPT_LIB="$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/$lib" timeout -k 10 120 python -u tools/band_one.py $rows 8 $tn >> $out 2>> gpurun_out/${TAG}_ab_band.err || exit $?
    done
  done
done
cat $out
