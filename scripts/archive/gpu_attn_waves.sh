#!/bin/bash
# Attention waves-per-block A/B: numerics under each setting, then ViT bench per setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for wv in 8,8,8 4,4,4; do
  ROCKET_ATTN_WAVES=$wv timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests_$wv.log 2>&1 || exit 1
done
for wv in 4,4,4 8,4,4 8,8,4 8,4,8 8,8,8 4,4,4; do
  echo -n "$wv " >> gpurun_out/attn_waves.txt
  ROCKET_ATTN_WAVES=$wv timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 >> gpurun_out/attn_waves.txt 2> gpurun_out/attn_waves.err || exit 1
done
