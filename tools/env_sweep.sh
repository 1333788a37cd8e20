#!/bin/bash
# C3 bench per environment setting: tools/env_sweep.sh "NAME:VAR=VAL ..." ...  (two rounds, alternating)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; vars=${spec#*:}
    env $vars timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/es_${name}_$i.json 2>/dev/null || exit $?
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/es_${name}_$i.json') if l.startswith('{')][-1]
print('%-10s' % '$name', d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
  done
done
