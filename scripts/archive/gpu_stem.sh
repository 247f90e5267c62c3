#!/bin/bash
# Fused stem BN+ReLU+maxpool: numerics, ResNet-50 bench, steady-state kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/stem_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/stem_rn50.json 2> gpurun_out/stem_rn50.err || exit 1
MODEL=resnet50 bash scripts/gpu_rn50_prof.sh
