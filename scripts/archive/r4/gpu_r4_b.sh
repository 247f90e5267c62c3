#!/bin/bash
# kernel tests (fp16 LeNet / ViT, LN, GELU, attention, CE), LeNet bf16/fp16 + ViT bf16/fp16 bench, xgemm ablation
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/kernels/test_fp16_vit.py \
  tests/kernels/test_ce_optim.py tests/kernels/test_fp16.py tests/kernels/test_linear_conv.py tests/kernels/test_norm.py \
  > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -3 gpurun_out/r4b_tests.log
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/r4b_lenet_bf16.json 2>gpurun_out/r4b_lenet_bf16.err || exit 1
timeout -k 10 120 python bench.py --mp fp16 --steps 300 --warmup 30 > gpurun_out/r4b_lenet_fp16.json 2>gpurun_out/r4b_lenet_fp16.err || exit 1
cat gpurun_out/r4b_lenet_bf16.json gpurun_out/r4b_lenet_fp16.json
timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/r4b_vit.json 2>gpurun_out/r4b_vit.err || exit 1
timeout -k 10 300 python bench.py --model vit_b16 --mp fp16 --steps 20 --warmup 5 > gpurun_out/r4b_vit_fp16.json 2>gpurun_out/r4b_vit_fp16.err || exit 1
cat gpurun_out/r4b_vit.json gpurun_out/r4b_vit_fp16.json
timeout -k 10 200 python -u bench/xgemm_dbg.py > gpurun_out/r4b_xgemm_dbg.jsonl 2>gpurun_out/r4b_xgemm_dbg.err || exit 1
cat gpurun_out/r4b_xgemm_dbg.jsonl
