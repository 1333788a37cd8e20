#!/bin/bash
# Kernel traces of several library builds on the C3 bench (one rocprofv3 run each), denoiser lines.
# Usage (on the box): tools/lib_kt.sh LIB...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "$@"; do
  t=$(basename $lib .so)
  VXPT_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/lkt_$t -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline > gpurun_out/lkt_$t.log 2>&1 || exit 1
  python tools/profsum.py gpurun_out/lkt_$t/run_results.db 30 | grep -E "^  .*(k_temporal|k_history_fix)" | sed "s/^/$t /"
  grep '^{' gpurun_out/lkt_$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t bench', d['value'], d['denoise_ms'])"
done
