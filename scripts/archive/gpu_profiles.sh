#!/bin/bash
# steady-state kernel profiles of all bench configs (kernel trace only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/summary_prof.txt
for m in lenet resnet18 resnet50 vit_b16; do
  steps=12; [ $m = lenet ] && steps=60
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_$m -o run -- python3 bench.py --model $m --steps $steps --warmup 5 > gpurun_out/prof_$m.log 2>&1; rc=$?
  echo "$m rc=$rc" >> gpurun_out/summary_prof.txt
  [ $rc -ne 0 ] && exit 1
done
exit 0
