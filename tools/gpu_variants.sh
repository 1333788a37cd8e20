#!/bin/bash
# GPU-box A/B of library variants: parity tests on the default library, then per variant a short
# bench and a kernel-trace profile.  Usage: tools/gpu_variants.sh TAG [name ...]  (libvxpt_<name>.so;
# "base" = libvxpt.so).  Each GPU step has its own time limit; a failing step ends the script.
TAG=${1:-v}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
PKG=real-time-path-tracing-voxel-blocks_amd
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tv_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv_$TAG.log
[ $rc -eq 0 ] || exit $rc
for name in base "$@"; do
    lib=$PKG/libvxpt.so; [ "$name" = base ] || lib=$PKG/libvxpt_$name.so
    VXPT_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 6 --no-cpu-baseline > gpurun_out/bv_${TAG}_$name.log 2>&1 || { echo "bench $name failed"; exit 1; }
    echo "$name $(python -c "import json,sys;d=json.loads(open('gpurun_out/bv_${TAG}_$name.log').read().strip().splitlines()[-1]);print('value',d['value'],'trace_ms',d['trace_ms'],'denoise_ms',d['denoise_ms'])")"
    cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
    VXPT_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/pv_${TAG}_$name -o run -- python bench.py --steps 3 --warmup 8 --no-cpu-baseline > gpurun_out/pv_${TAG}_$name.log 2>&1 || { echo "prof $name failed"; exit 1; }
    python tools/profsum.py gpurun_out/pv_${TAG}_$name/run_results.db 40 > gpurun_out/pv_${TAG}_$name.txt
done
