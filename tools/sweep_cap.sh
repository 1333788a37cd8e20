#!/bin/bash
# Iteration-cap sweep of the straggler traversal (GPU box): tests, then bench per (cap, cap2).
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tsw.log 2>&1; echo pytest rc=$?; tail -2 gpurun_out/tsw.log
for cc in ${CAPS:-6:0 4:6 5:8 6:8 6:12 8:8}; do
  c=${cc%%:*}; c2=${cc##*:}
  VXPT_ITER_CAP=$c VXPT_ITER_CAP2=$c2 timeout -k 10 100 python bench.py --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/sw_${c}_${c2}.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sw_${c}_${c2}.log').read().strip().splitlines()[-1]);print('cap $c $c2', d['value'],d['trace_ms'])"
done
