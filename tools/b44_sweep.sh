#!/bin/bash
# The 4/4-bounce C3 reading under tuning variants, two alternating rounds.  Usage (on the box):
#   tools/b44_sweep.sh "NAME:field=v,..." ...
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  for spec in "$@"; do
    vals=${spec#*:}; args=""
    for kv in ${vals//,/ }; do args="$args --tune $kv"; done
    timeout -k 10 200 python -u bench.py --bounces 4/4 --steps 6 --warmup 3 --no-cpu-baseline $args > /tmp/b44.json 2>/dev/null || exit $?
    python -c "
import json; d=[json.loads(l) for l in open('/tmp/b44.json') if l.startswith('{')][-1]
print('%-10s' % '${spec%%:*}', d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
  done
done
