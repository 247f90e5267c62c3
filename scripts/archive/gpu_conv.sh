#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in FAST NORMAL; do
  MIOPEN_FIND_MODE=$mode timeout -k 10 300 python bench/conv_probe.py > gpurun_out/conv_$mode.jsonl 2> gpurun_out/conv_$mode.err; echo "$mode rc=$?" >> gpurun_out/summary_conv.txt
done
MIOPEN_FIND_MODE=FAST timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r18 -o run -- python3 bench.py --model resnet18 --no-graph --steps 5 --warmup 3 > gpurun_out/prof_r18.log 2>&1; echo "prof rc=$?" >> gpurun_out/summary_conv.txt
