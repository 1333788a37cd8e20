cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 480 --timeout-method thread -m gpu tests/test_gpu_frames_spp.py -k steady > gpurun_out/steady_default.log 2>&1
rc=$?; echo "default rc=$rc"; [ $rc -le 1 ] || exit $rc
VXPT_LIB="$GRAFT_REPO_ROOT/real-time-path-tracing-voxel-blocks_amd/libvxpt_exact.so" timeout -k 10 500 python -u -m pytest -v -s --timeout 480 --timeout-method thread -m gpu tests/test_gpu_frames_spp.py -k steady > gpurun_out/steady_exact.log 2>&1
rc=$?; echo "exact rc=$rc"; [ $rc -le 1 ] || exit $rc
bash tools/gpu_trace_roofline.sh r06
