#!/bin/bash
# BN finalize launches: numerics, ResNet benches, ResNet-18 trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_iconv.py tests/kernels/test_norm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fin_tests.log 2>&1 || exit 1
for m in resnet18 resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 >> gpurun_out/fin_bench.jsonl 2> gpurun_out/fin_bench.err || exit 1
done
MODELS="resnet18" bash scripts/gpu_prof_models.sh
