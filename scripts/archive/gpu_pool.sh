#!/bin/bash
# Stem pool kernels (32-bit index math): numerics, ResNet-50 bench, kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pool_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/pool_rn50.json 2> gpurun_out/pool_rn50.err || exit 1
MODEL=resnet50 bash scripts/gpu_rn50_prof.sh
