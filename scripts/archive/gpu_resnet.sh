#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/summary_resnet.txt
for m in resnet18 resnet50; do
  timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bench_${m}_graph.json 2> gpurun_out/bench_${m}_graph.err; rc=$?; echo "$m graph rc=$rc" >> gpurun_out/summary_resnet.txt
  [ $rc -ne 0 ] && exit 1
  timeout -k 10 400 python bench.py --model $m --no-graph --steps 20 --warmup 5 > gpurun_out/bench_${m}_eager.json 2> gpurun_out/bench_${m}_eager.err; rc=$?; echo "$m eager rc=$rc" >> gpurun_out/summary_resnet.txt
  [ $rc -ne 0 ] && exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --no-graph --steps 10 --warmup 5 > gpurun_out/prof_r50.log 2>&1; echo "prof rc=$?" >> gpurun_out/summary_resnet.txt
