#!/bin/bash
# Round 3: native stem + attention layout: kernel tests, branch probe, 1-GPU benches of every model
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/kernels/test_iconv.py tests/kernels/test_norm.py tests/gpu/test_models.py \
  > gpurun_out/r3_b_tests.log 2>&1 || { tail -40 gpurun_out/r3_b_tests.log; exit 1; }
tail -3 gpurun_out/r3_b_tests.log
timeout -k 10 120 python bench/graph_branch_probe.py > gpurun_out/r3_branch_probe.json 2>gpurun_out/r3_branch_probe.err || exit 1
cat gpurun_out/r3_branch_probe.json
for m in lenet resnet18 resnet50 vit_b16; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r3_b_$m.json 2>gpurun_out/r3_b_$m.err || exit 1
  cat gpurun_out/r3_b_$m.json
done
