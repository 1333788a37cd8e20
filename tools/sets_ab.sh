#!/bin/bash
# bench with 2 and 3 wavefront state sets (VXPT_SETS), alternating, on one box
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  for k in 2 3; do
    VXPT_SETS=$k timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/sets${k}_$i.log 2>&1 || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/sets${k}_$i.log') if l.startswith('{')][-1]
print('sets $k', d['value'], d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
  done
done
