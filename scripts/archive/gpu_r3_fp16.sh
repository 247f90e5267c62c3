#!/bin/bash
# fp16 autocast: the split-K slab combine test, then the fp16 ViT-B/16 bench that faulted before the fix
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_mgemm.py tests/kernels/test_amp.py -m gpu > gpurun_out/fp16_tests.log 2>&1 || { tail -30 gpurun_out/fp16_tests.log; exit 1; }
tail -2 gpurun_out/fp16_tests.log
timeout -k 10 300 python bench.py --model vit_b16 --mp fp16 --steps 10 --warmup 3 > gpurun_out/fp16_vit.json 2> gpurun_out/fp16_vit.err || { tail -20 gpurun_out/fp16_vit.err; exit 1; }
cat gpurun_out/fp16_vit.json
