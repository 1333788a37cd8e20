set -o pipefail
bash tools/tune_sweep.sh base:overlap=1 p1:stream_priority=1 p2:stream_priority=2 > gpurun_out/prio.txt 2>&1 || exit $?
bash tools/lib_ab.sh cur=cur rb=real-time-path-tracing-voxel-blocks_amd/libvxpt_rb.so rb3=real-time-path-tracing-voxel-blocks_amd/libvxpt_rb3.so > gpurun_out/rb_ab.txt 2>&1 || exit $?
VXPT_LIB=real-time-path-tracing-voxel-blocks_amd/libvxpt_rb.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_frames_spp.py > gpurun_out/rb_tests.log 2>&1; echo "rb tests rc=$?"
bash tools/gpu_batch.sh tests
