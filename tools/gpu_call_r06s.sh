#!/bin/bash
# Round 6: k_closest in XCD-local panels (xcd_order 2) on the camera-ray-only C2 line and on 1080p bands.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r06s_c2.txt; : > $out
for i in 1 2; do
  for t in 0 2; do
    timeout -k 10 200 python bench.py --primary-only --no-cpu-baseline --steps 50 --tune xcd_order=$t > gpurun_out/r06s_c2_${t}_${i}.log 2>&1 || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06s_c2_${t}_${i}.log') if l.startswith('{')][-1]
print('xcd_order=$t', d['value'], d['ms_per_step'])" >> $out
  done
done
cat $out
bash tools/gpu_call_ab_band.sh r06s libvxpt.so libvxpt.so@xcd_order=2
