set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_frames_spp.py tests/test_bands.py > gpurun_out/hf_tests.log 2>&1 && bash tools/chain_diag.sh hfc
