#!/bin/bash
# A/B of several library builds / tunings on the C3 bench: every kernel alone (--tune overlap=0) under a
# kernel trace -- the denoiser chain's kernels over the last 4 frames (tools/chain_kt.py) -- then the
# default bench of each, interleaved, twice.  Usage (on the box): tools/ab_multi.sh TAG VARIANT...
# where VARIANT = LIB[@field=value[@field=value...]] (the fields go to bench.py --tune).
TAG=$1; shift
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tunes() { local IFS=@; set -- $1; shift; for t in "$@"; do printf -- "--tune %s " "$t"; done; }
n=0
for v in "$@"; do
  n=$((n+1)); lib=${v%%@*}; tn=$(tunes "$v")
  VXPT_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/${TAG}_$n -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline --tune overlap=0 $tn > gpurun_out/${TAG}_${n}_kt.log 2>&1 || exit 1
  python tools/chain_kt.py gpurun_out/${TAG}_$n/run_results.db > gpurun_out/${TAG}_${n}_chain.txt
  python tools/profsum.py gpurun_out/${TAG}_$n/run_results.db > gpurun_out/${TAG}_${n}_kt.txt
  echo "== $n $v"; cat gpurun_out/${TAG}_${n}_chain.txt
done
for i in 1 2; do
  n=0
  for v in "$@"; do
    n=$((n+1)); lib=${v%%@*}; tn=$(tunes "$v")
    VXPT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 $tn > gpurun_out/${TAG}_${n}_b$i.log 2>&1 || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/${TAG}_${n}_b$i.log') if l.startswith('{')][-1]
print('$n', '$v'.split('/')[-1], d['value'], d['ms_per_step'], d['trace_ms'], d['denoise_ms'], d['roofline_chain_alone']['avg_duration_ms'])"
  done
done
