#!/bin/bash
# BatchNorm backward reduction in the conv dgrad epilogue: numerics, ResNet benches (fused vs
# ROCKET_BN_BWD_FUSE=0), ResNet-50 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_iconv.py tests/kernels/test_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bnb_tests.log 2>&1 || exit 1
for m in resnet50 resnet18; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bnb_$m.json 2> gpurun_out/bnb_$m.err || exit 1
  ROCKET_BN_BWD_FUSE=0 timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bnb_${m}_off.json 2> gpurun_out/bnb_${m}_off.err || exit 1
done
MODEL=resnet50 bash scripts/gpu_rn50_prof.sh
