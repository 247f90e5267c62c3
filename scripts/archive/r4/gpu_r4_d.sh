#!/bin/bash
# optimizer/shadow + LeNet tests, LeNet bf16/fp16 bench, ViT bf16 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_ce_optim.py \
  tests/kernels/test_fp16.py tests/kernels/test_linear_conv.py tests/kernels/test_amp.py > gpurun_out/r4d_tests.log 2>&1 \
  || { tail -40 gpurun_out/r4d_tests.log; exit 1; }
tail -2 gpurun_out/r4d_tests.log
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/r4d_lenet_bf16.json 2>gpurun_out/r4d_lenet_bf16.err || exit 1
timeout -k 10 120 python bench.py --mp fp16 --steps 300 --warmup 30 > gpurun_out/r4d_lenet_fp16.json 2>gpurun_out/r4d_lenet_fp16.err || exit 1
cat gpurun_out/r4d_lenet_bf16.json gpurun_out/r4d_lenet_fp16.json | cut -c1-400
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4d_vit -o run -- python3 $R/bench.py --model vit_b16 --steps 8 --warmup 3 > $R/gpurun_out/r4d_vit_trace.log 2>&1 || { tail -20 $R/gpurun_out/r4d_vit_trace.log; exit 1; }
cd $R
f=$(find gpurun_out/r4d_vit -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ViT-B/16 bs128 bf16 step (round 4), rocprofv3 kernel trace" > gpurun_out/r4_vit_b16_kernels.md
rm -rf gpurun_out/r4d_vit
head -40 gpurun_out/r4_vit_b16_kernels.md
