#!/bin/bash
# A/B of the LDS-windowed temporal accumulation (VXPT_TA_LDS) and its occupancy variant on the C3
# bench: denoiser-chain HIP-event time of the default bench, then a kernel trace of each setting.
# Usage (on the box): tools/ta_ab.sh [extra libs ...]
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ta_${tag}.log 2>&1 || { echo "bench $tag failed"; tail gpurun_out/ta_${tag}.log; exit 1; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ta_${tag}.log') if l.startswith('{')][-1]
print('$tag', d['value'], d['ms_per_step'], d['trace_ms'], d['denoise_ms'])"
}
for i in 1 2; do
  run lds$i VXPT_TA_LDS=1
  run glb$i VXPT_TA_LDS=0
  for lib in "$@"; do run $(basename $lib .so)$i VXPT_LIB=$lib; done
done
for tag in lds glb; do
  v=1; [ $tag = glb ] && v=0
  VXPT_TA_LDS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/takt_$tag -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline > gpurun_out/takt_${tag}.log 2>&1 || exit 1
  python tools/profsum.py gpurun_out/takt_$tag/run_results.db 30 | grep -E "k_temporal|k_history|k_atrous|k_firefly" | sed "s/^/$tag /"
done
