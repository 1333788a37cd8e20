#!/bin/bash
# One band's frame time (a rank of the 8-band 1080p partition, rows 408-544, and an 8-row band) under
# tuning variants, on top of bench.band_tuning's banded defaults.  Usage (on the box):
#   tools/band_tune.sh "NAME:field=v,..." ...
cd "$GRAFT_REPO_ROOT" || exit 1
for spec in "$@"; do
  vals=${spec#*:}; args="--tune state_sets=3 --tune front_streams=3"
  for kv in ${vals//,/ }; do args="$args --tune $kv"; done
  for rows in "408 544" "408 416"; do
    echo "${spec%%:*} $(timeout -k 10 100 python tools/band_kt.py $rows $args --frames 10)" || exit 1
  done
done
