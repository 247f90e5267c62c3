#!/bin/bash
# LN-backward bias accumulation (BiasLink into persistent grads), fp16 loss scale folded into the
# fused LeNet cross-entropy, skip flags via a host-mapped ring: numerics, LeNet / ViT benches (bf16, fp16), the current ViT kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py \
  tests/kernels/test_fp16_vit.py tests/kernels/test_fp16.py tests/kernels/test_amp.py \
  tests/kernels/test_ce_optim.py tests/gpu/test_launcher_gpu.py tests/gpu/test_p2p.py > gpurun_out/r4j_tests.log 2>&1 || { tail -30 gpurun_out/r4j_tests.log; exit 1; }
tail -2 gpurun_out/r4j_tests.log
timeout -k 10 200 python bench.py --mp fp16 > gpurun_out/r4j_lenet_fp16.json 2>gpurun_out/r4j_lenet_fp16.err || exit 1
timeout -k 10 200 python bench.py > gpurun_out/r4j_lenet_bf16.json 2>gpurun_out/r4j_lenet_bf16.err || exit 1
cut -c1-330 gpurun_out/r4j_lenet_fp16.json gpurun_out/r4j_lenet_bf16.json
timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/r4j_vit.json 2>gpurun_out/r4j_vit.err || exit 1
timeout -k 10 300 python bench.py --model vit_b16 --mp fp16 --steps 20 --warmup 5 > gpurun_out/r4j_vit_fp16.json 2>gpurun_out/r4j_vit_fp16.err || exit 1
cut -c1-200 gpurun_out/r4j_vit.json gpurun_out/r4j_vit_fp16.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4j_vit -o run -- python3 $R/bench.py --model vit_b16 --steps 8 --warmup 3 > $R/gpurun_out/r4j_vit_trace.log 2>&1 || { tail -20 $R/gpurun_out/r4j_vit_trace.log; exit 1; }
cd $R
f=$(find gpurun_out/r4j_vit -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ViT-B/16 bs128 bf16 step (round 4, final), rocprofv3 kernel trace" > gpurun_out/r4_vit_b16_kernels_final.md
rm -rf gpurun_out/r4j_vit
head -40 gpurun_out/r4_vit_b16_kernels_final.md
