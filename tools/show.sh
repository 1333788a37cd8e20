#!/bin/bash
# summarise a tools/gpu_check.sh run: tools/show.sh TAG
T=$1
tail -3 gpurun_out/call_$T.txt 2>/dev/null
tail -1 gpurun_out/bench_$T.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ('value','ms_per_step','trace_ms','denoise_ms','trace_mpaths_s')}, 'roofline', d['roofline']['frac'])"
echo "passed: $(grep -c PASSED gpurun_out/gpu_tests_$T.log)"; grep FAILED gpurun_out/gpu_tests_$T.log | head
python tools/profsum.py gpurun_out/prof_$T/run_results.db ${2:-16} | tail -${2:-16}
