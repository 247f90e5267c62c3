#!/bin/bash
# fp16 LeNet: non-finite check folded into the weight-gradient launch; numerics, bench, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_fp16.py \
  tests/kernels/test_amp.py tests/kernels/test_ce_optim.py tests/kernels/test_linear_conv.py tests/gpu/test_launcher_gpu.py > gpurun_out/r4l_tests.log 2>&1 || { tail -30 gpurun_out/r4l_tests.log; exit 1; }
tail -2 gpurun_out/r4l_tests.log
timeout -k 10 200 python bench.py --mp fp16 > gpurun_out/r4l_lenet_fp16.json 2>gpurun_out/r4l_lenet_fp16.err || exit 1
timeout -k 10 200 python bench.py --mp fp16 > gpurun_out/r4l_lenet_fp16b.json 2>gpurun_out/r4l_lenet_fp16b.err || exit 1
timeout -k 10 200 python bench.py > gpurun_out/r4l_lenet_bf16.json 2>gpurun_out/r4l_lenet_bf16.err || exit 1
cut -c1-330 gpurun_out/r4l_lenet_fp16.json gpurun_out/r4l_lenet_fp16b.json gpurun_out/r4l_lenet_bf16.json
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4l_lf16 -o run -- python3 $R/bench.py --mp fp16 --steps 40 --warmup 10 > $R/gpurun_out/r4l_lf16.log 2>&1 || { tail -20 $R/gpurun_out/r4l_lf16.log; exit 1; }
cd $R
f=$(find gpurun_out/r4l_lf16 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 20 --marker mlp3_wgrad --title "LeNet bs1024 fp16 step (round 4), kernel trace" > gpurun_out/r4_lenet_fp16_kernels.md || true
rm -rf gpurun_out/r4l_lf16
head -14 gpurun_out/r4_lenet_fp16_kernels.md
