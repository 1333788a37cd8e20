#!/bin/bash
# trace time per (VXPT_BRICK_STEPS, VXPT_ITER_CAP) on the C3 bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  b=${v%%:*}; c=${v##*:}
  VXPT_BRICK_STEPS=$b VXPT_ITER_CAP=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/ws_${b}_${c}.json 2>/dev/null || exit $?
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ws_${b}_${c}.json') if l.startswith('{')][-1]
print('brick steps $b cap $c', d['trace_ms'], d['ms_per_step'])"
done
