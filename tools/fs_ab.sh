export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "tuning or pipelined or overlapped" > gpurun_out/fs_tests.log 2>&1; echo trc=$?; tail -2 gpurun_out/fs_tests.log
bash tools/tune_sweep.sh "def:overlap=1" "fs2:front_streams=2" "fs2s3:front_streams=2,state_sets=3" || exit 1
for t in "" "--tune front_streams=2" "--tune front_streams=2 --tune state_sets=3"; do timeout -k 10 100 python tools/band_kt.py 408 544 $t || exit 1; timeout -k 10 100 python tools/band_kt.py 408 416 $t || exit 1; done
