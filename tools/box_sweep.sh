#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 8:8 8:16 8:32 8:64 16:16 16:64 4:64 32:64; do
  c=${v%%:*}; u=${v##*:}
  VXPT_BOX_CAP=$c VXPT_BOX_CAP_UP=$u timeout -k 10 200 python -u bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/bx_${c}_${u}.json 2>/dev/null || exit $?
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/bx_${c}_${u}.json') if l.startswith('{')][-1]
print('cap $c up $u', d['trace_ms'], d['ms_per_step'])"
done
