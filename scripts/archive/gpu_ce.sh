#!/bin/bash
# LeNet fused-CE check: kernel tests + graph bench + steady-state kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/kernels/test_linear_conv.py tests/gpu -q -m gpu -x > gpurun_out/t.log 2>&1 || { tail -5 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_lenet -o run -- python3 $R/bench.py --steps 60 --warmup 5 > $R/gpurun_out/prof_lenet.log 2>&1 || exit 1
cd $R && python bench/summarize_trace.py $(ls gpurun_out/prof_lenet/*/run_kernel_trace.csv gpurun_out/prof_lenet/run_kernel_trace.csv 2>/dev/null | head -1) --steps 20 --title "LeNet graph step" > gpurun_out/lenet_steady.md
cat gpurun_out/lenet_steady.md
