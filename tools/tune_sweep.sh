#!/bin/bash
# C3 bench per schedule setting (vxpt_tuning through bench.py --tune), two rounds alternating:
# tools/tune_sweep.sh "NAME:field=val,field=val" ...   e.g. "cap4:iter_cap=4" "noov:overlap=0"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; vals=${spec#*:}
    args=""
    for kv in ${vals//,/ }; do args="$args --tune $kv"; done
    timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > gpurun_out/ts_${name}_$i.json 2>/dev/null || exit $?
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ts_${name}_$i.json') if l.startswith('{')][-1]
print('%-10s' % '$name', d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
  done
done
