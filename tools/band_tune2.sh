#!/bin/bash
# One band's frame time for several band sizes under tuning variants, two alternating rounds, on top of
# bench.band_tuning's banded defaults for the band's size.  Usage (on the box):
#   tools/band_tune2.sh "Y0 Y1;Y0 Y1;..." "NAME:field=v,..." ...
cd "$GRAFT_REPO_ROOT" || exit 1
IFS=';' read -ra BANDS <<< "$1"; shift
for i in 1 2; do
  for rows in "${BANDS[@]}"; do
    read -r y0 y1 <<< "$rows"
    fs=2; [ $(( (y1 - y0) * 1920 )) -lt 700000 ] && fs=3
    for spec in "$@"; do
      vals=${spec#*:}; args="--tune state_sets=3 --tune front_streams=$fs"
      for kv in ${vals//,/ }; do args="$args --tune $kv"; done
      echo "${spec%%:*} $(timeout -k 10 100 python tools/band_kt.py $y0 $y1 $args --frames 10)" || exit 1
    done
  done
done
