#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python bench/lenet_timeline.py > gpurun_out/r3_lenet_timeline.jsonl 2> gpurun_out/r3_lenet_timeline.err || exit 1
cat gpurun_out/r3_lenet_timeline.jsonl | head -c 3000
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_lenet -o run -- python3 $R/bench.py --steps 200 --warmup 20 > $R/gpurun_out/prof_lenet.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/prof_lenet -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 50 --title "LeNet bs1024 fused step - rocprofv3 --kernel-trace" > gpurun_out/r3_lenet_kernels.md; rc=$?
rm -rf gpurun_out/prof_lenet
cat gpurun_out/r3_lenet_kernels.md
exit $rc
