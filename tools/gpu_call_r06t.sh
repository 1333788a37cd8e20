#!/bin/bash
# Round 6: bands -- fewer straggler launches (a high iteration cap) and smaller straggler grids.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_call_ab_band.sh r06t libvxpt.so libvxpt.so@iter_cap=12 libvxpt.so@iter_cap=1024@iter_cap2=0 \
  libvxpt.so@resume_wg_per_cu=4 libvxpt.so@resume_wg_per_cu=8
