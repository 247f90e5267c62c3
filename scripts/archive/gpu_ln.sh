#!/bin/bash
# LayerNorm backward: numerics, ViT bench x2, kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py tests/gpu/test_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ln_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 >> gpurun_out/ln_vit.jsonl 2> gpurun_out/ln_vit.err || exit 1
done
MODELS="vit_b16" bash scripts/gpu_prof_models.sh
