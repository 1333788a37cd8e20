#!/bin/bash
# Kernel-trace averages of the C3 bench with kernels one at a time, per tuning setting:
# tools/tune_kt.sh "NAME:field=v,..." ...   -> gpurun_out/tkt_NAME.txt
export TMPDIR=/tmp; cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1; mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; vals=${spec#*:}; args="--tune overlap=0"
  for kv in ${vals//,/ }; do args="$args --tune $kv"; done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/tkt_$name -o run -- python bench.py --steps 4 --warmup 8 --no-cpu-baseline $args > gpurun_out/tkt_$name.log 2>&1 || exit 1
  python tools/profsum.py gpurun_out/tkt_$name/run_results.db > gpurun_out/tkt_$name.txt
  echo "== $name"; grep -E "k_closest|k_shade|k_restir|k_finish|k_nee" gpurun_out/tkt_$name.txt
done
