export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/kt_noov -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline --tune overlap=0 > gpurun_out/kt_noov.log 2>&1 || { echo "noov failed"; exit 1; }
python tools/profsum.py gpurun_out/kt_noov/run_results.db 120 > gpurun_out/kt_noov.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/kt_band -o run -- python tools/band_kt.py 408 544 > gpurun_out/kt_band.log 2>&1 || { echo "band failed"; exit 1; }
python tools/timeline.py gpurun_out/kt_band/run_results.db 160 > gpurun_out/kt_band_timeline.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/kt_bandnoov -o run -- python tools/band_kt.py 408 544 --tune overlap=0 > gpurun_out/kt_bandnoov.log 2>&1 || { echo "band noov failed"; exit 1; }
python tools/profsum.py gpurun_out/kt_bandnoov/run_results.db 120 > gpurun_out/kt_bandnoov.txt
python tools/timeline.py gpurun_out/kt_bandnoov/run_results.db 160 > gpurun_out/kt_bandnoov_timeline.txt
for y in 8 32 136 272; do timeout -k 10 100 python tools/band_kt.py 408 $((408+y)) >> gpurun_out/band_sizes.log 2>&1 || exit 1; done
echo done
