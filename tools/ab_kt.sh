#!/bin/bash
# A/B of two library builds on the C3 bench, kernels one at a time (--tune overlap=0) under a kernel
# trace, plus the default (overlapped) bench of each.  Usage (on the box): tools/ab_kt.sh OLD.so NEW.so
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for tag in old new; do
  lib=$1; [ $tag = new ] && lib=$2
  VXPT_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/ab_$tag -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline --tune overlap=0 > gpurun_out/ab_${tag}_kt.log 2>&1 || exit 1
  python tools/profsum.py gpurun_out/ab_$tag/run_results.db 30 > gpurun_out/ab_${tag}_kt.txt
done
for i in 1 2; do
  for tag in old new; do
    lib=$1; [ $tag = new ] && lib=$2
    VXPT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_${tag}_b$i.log 2>&1 || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab_${tag}_b$i.log') if l.startswith('{')][-1]
print('$tag', d['value'], d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
  done
done
