#!/bin/bash
# new kernels (norm/act) + model-level tests + first ResNet/ViT benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/kernels/test_norm.py tests/gpu/test_models.py -m gpu -q > gpurun_out/pytest_models.log 2>&1; echo "pytest rc=$?" > gpurun_out/summary.txt
for m in resnet18 resnet50 vit_b16; do
  timeout -k 10 400 python bench.py --model $m --no-graph --steps 20 --warmup 5 > gpurun_out/bench_${m}_eager.json 2> gpurun_out/bench_${m}_eager.err; rc=$?; echo "$m eager rc=$rc" >> gpurun_out/summary.txt
  [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit 1
  timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bench_${m}_graph.json 2> gpurun_out/bench_${m}_graph.err; rc=$?; echo "$m graph rc=$rc" >> gpurun_out/summary.txt
  [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit 1
done
exit 0
