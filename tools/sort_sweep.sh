#!/bin/bash
# bench trace time per VXPT_SORT mode (ray queues grouped by direction class)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in 0 1 2 0; do
  VXPT_SORT=$m timeout -k 10 200 python -u bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/sort_$m.json 2>/dev/null || exit $?
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/sort_$m.json') if l.startswith('{')][-1]
print('sort $m', d['trace_ms'], d['ms_per_step'])"
done
