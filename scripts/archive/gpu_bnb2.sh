#!/bin/bash
# BN-backward reduction in the LDS-staged dgrad epilogue: numerics, A/B benches (ROCKET_BN_BWD_FUSE=1 vs 0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_iconv.py tests/kernels/test_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bnb2_tests.log 2>&1 || exit 1
for m in resnet50 resnet18; do
  for f in 1 0 1; do
    ROCKET_BN_BWD_FUSE=$f timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 >> gpurun_out/bnb2_$m.jsonl 2> gpurun_out/bnb2_$m.err || exit 1
  done
done
bash scripts/gpu_bnb_calls.sh
