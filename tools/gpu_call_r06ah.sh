#!/bin/bash
# Round 6: the later path segments' queues (4/4 bounces) on the walk ladder too (build libvxpt_ll.so,
# -DVX_LATER_LADDER=1) against the default (8 more iterations, then pieces): 4/4 bench, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 env VXPT_LIB=$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt_ll.so python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "later_segment or tuning_changes_no_result" > gpurun_out/r06ah_tests.log 2>&1 || { tail -30 gpurun_out/r06ah_tests.log; exit 1; }
tail -1 gpurun_out/r06ah_tests.log
for i in 1 2 3; do
  for lib in libvxpt.so libvxpt_ll.so; do
    VXPT_LIB=$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/$lib timeout -k 10 200 python -u bench.py --bounces 4/4 --no-cpu-baseline --steps 10 --warmup 4 > gpurun_out/r06ah_${lib}_$i.json 2>/dev/null || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06ah_${lib}_$i.json') if l.startswith('{')][-1]
print('$lib', d['value'], d['ms_per_step'])"
  done
done
