#!/bin/bash
# Round 3: overlapped DP capture tests + branch concurrency probe + quick LeNet bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/gpu/test_dp_overlap.py tests/gpu/test_native_runtime.py tests/gpu/test_launch_list.py \
  tests/gpu/test_p2p.py tests/kernels/test_amp.py tests/kernels/test_iconv.py tests/gpu/test_ddp_graph.py \
  > gpurun_out/r3_dp_tests.log 2>&1 || { tail -40 gpurun_out/r3_dp_tests.log; exit 1; }
tail -5 gpurun_out/r3_dp_tests.log
timeout -k 10 120 python bench/graph_branch_probe.py > gpurun_out/r3_branch_probe.json 2>gpurun_out/r3_branch_probe.err || exit 1
cat gpurun_out/r3_branch_probe.json
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_lenet.json 2>gpurun_out/r3_lenet.err || exit 1
cat gpurun_out/r3_lenet.json
