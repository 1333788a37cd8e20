#!/bin/bash
# Alternating A/B of library builds on the C3 bench (pipelined and per-call frame loops).
# Usage (on the box): tools/lib_ab.sh NAME=LIB[:bench args] ...   (LIB "cur" = the tree's libvxpt.so)
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; args=""
    [ "$rest" != "$lib" ] && args=${rest#*:}
    [ "$lib" = cur ] && lib=real-time-path-tracing-voxel-blocks_amd/libvxpt.so
    for mode in "" "--frame-calls"; do
      VXPT_LIB=$lib timeout -k 10 100 python bench.py --steps 20 --warmup 6 --no-cpu-baseline $mode $args > /tmp/ab.json 2>/dev/null || { echo "$name failed"; exit 1; }
      python -c "
import json; d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1])
print('%-10s %-13s %.4f %.4f %.4f' % ('$name', '${mode:-pipelined}', d['ms_per_step'], d['trace_ms'], d['denoise_ms']))"
    done
  done
done
