#!/bin/bash
# Attention: 8-wave blocks with and without the 2-blocks-per-CU register bound (82), ViT bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
ROCKET_ATTN_WAVES=82,82,82 timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn2_tests.log 2>&1 || exit 1
for wv in 8,8,8 82,8,8 8,82,8 8,8,82 8,82,82 8,8,8; do
  echo -n "$wv " >> gpurun_out/attn_waves2.txt
  ROCKET_ATTN_WAVES=$wv timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 >> gpurun_out/attn_waves2.txt 2> gpurun_out/attn_waves2.err || exit 1
done
