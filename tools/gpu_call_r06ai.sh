#!/bin/bash
# Round 6: traversal occupancy bounds on the final tree (build variants: straggler resume 7 / 8 waves,
# closest-hit resume 7, k_queue 8), tools/ab_multi.sh.
cd "$GRAFT_REPO_ROOT" || exit 1
D=$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd
bash tools/ab_multi.sh r06ai $D/libvxpt.so $D/libvxpt_r7.so $D/libvxpt_r8.so $D/libvxpt_rc7.so $D/libvxpt_q8.so
