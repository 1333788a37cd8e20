#!/bin/bash
# denoiser variants (environment knobs): per-kernel times from a kernel-trace pass + the bench's chain time
# Usage (on the box): tools/dn_sweep.sh "NAME:VAR=VAL ..." ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 200 python -u bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/dn_$name.json 2>/dev/null || exit $?
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/dn_$name.json') if l.startswith('{')][-1]
print('$name', 'denoise_ms', d['denoise_ms'], 'trace_ms', d['trace_ms'])"
  env $vars timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/dnk_$name -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline > /dev/null 2>&1 || exit $?
  python tools/profsum.py gpurun_out/dnk_$name/run_results.db | grep -E "k_temporal|k_history|k_atrous|k_firefly" 
done
