#!/bin/bash
# C3 bench per (VXPT_PERSIST workgroups per CU : VXPT_REFILL idle lanes); 0 = iteration-capped k_queue + k_resume
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  p=${v%%:*}; r=${v##*:}
  VXPT_PERSIST=$p VXPT_REFILL=$r timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ps_${p}_${r}.json 2>/dev/null || exit $?
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ps_${p}_${r}.json') if l.startswith('{')][-1]
print('persist $p refill $r', d['trace_ms'], d['ms_per_step'])"
done
