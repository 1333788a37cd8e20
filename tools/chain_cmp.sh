export TMPDIR=/tmp; cd /tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in pipe calls; do
  a=""; [ $m = calls ] && a="--frame-calls"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/cc_$m -o run -- python bench.py --steps 8 --warmup 8 --no-cpu-baseline $a > gpurun_out/cc_$m.log 2>&1 || exit 1
done
echo ok
