#!/bin/bash
# C2 (primary-only) bench per environment setting: tools/c2_sweep.sh "NAME:VAR=VAL ..." ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; vars=${spec#*:}
    env $vars timeout -k 10 200 python -u bench.py --primary-only --no-cpu-baseline --steps 50 > gpurun_out/c2s_${name}_$i.json 2>/dev/null || exit $?
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/c2s_${name}_$i.json') if l.startswith('{')][-1]
print('c2 %-8s' % '$name', d['value'], d['ms_per_step'])"
  done
done
