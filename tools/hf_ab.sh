#!/bin/bash
# History-fix split sweep (VXPT_HF_SPLIT) on the C3 bench: chain time of the default bench and the
# steady-state k_history_fix duration from a kernel trace.  Usage (on the box): tools/hf_ab.sh
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  [ -n "$1" ] && { VXPT_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/hf_lib.log 2>&1 && python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/hf_lib.log') if l.startswith('{')][-1]
print('lib', d['value'], d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"; }
  for s in 1 2 4 8; do
    VXPT_HF_SPLIT=$s timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/hf_$s.log 2>&1 || { echo "bench $s failed"; exit 1; }
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/hf_$s.log') if l.startswith('{')][-1]
print('split $s', d['value'], d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
  done
done
for s in 1 4; do
  VXPT_HF_SPLIT=$s timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/hfkt_$s -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline > gpurun_out/hfkt_$s.log 2>&1 || exit 1
  python tools/profsum.py gpurun_out/hfkt_$s/run_results.db 30 | grep -E "k_history_fix" | sed "s/^/split $s /"
done
if [ -n "$1" ]; then
  VXPT_LIB=$1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/hfkt_lib -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline > gpurun_out/hfkt_lib.log 2>&1 || exit 1
  python tools/profsum.py gpurun_out/hfkt_lib/run_results.db 30 | grep -E "k_history_fix" | sed "s/^/lib /"
fi
