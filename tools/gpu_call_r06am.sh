#!/bin/bash
# Round 6: the empty-box growth order (build variants VX_BOX_ORDER: 1 = y first in the upward octants,
# 2 = x, y, z; default x, z, y), C3 bench, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
D=$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd
for r in 1 2 3; do
  for lib in libvxpt.so libvxpt_bo1.so libvxpt_bo2.so; do
    VXPT_LIB=$D/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06am_${lib}_$r.json 2>/dev/null || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06am_${lib}_$r.json') if l.startswith('{')][-1]
print('%-16s' % '$lib', d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
  done
done
