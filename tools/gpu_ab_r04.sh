#!/bin/bash
# Round-4 A/B call: the tree's library against an experiment build (alternating C3 benches), then
# every GPU test.  Usage (on the box): tools/gpu_ab_r04.sh NAME=LIB ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/lib_ab.sh cur=cur "$@" > gpurun_out/ab.txt 2>&1 || exit $?
bash tools/gpu_batch.sh tests
