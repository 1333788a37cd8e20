#!/bin/bash
# Round 6: the walk schedule of an 8-band 1080p band re-swept with the sky exit and iter_cap 5
# (tools/gpu_call_ab_band.sh: three bands, two interleaved runs each).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_call_ab_band.sh r06p libvxpt.so libvxpt.so@iter_cap=4 libvxpt.so@iter_cap=7 \
  libvxpt.so@iter_cap2=5 libvxpt.so@iter_cap2=12 libvxpt.so@resume_split=8 libvxpt.so@restir_waves=4
