#!/bin/bash
# LeNet headline bench, 3 repeats (graph path)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 3000 --warmup 30 > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err || exit 1
  cat gpurun_out/bench_$i.json
done
