#!/bin/bash
# Round 3: overlapped DP capture tests, attention layout, branch concurrency probe, quick benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/gpu/test_ddp_graph.py tests/gpu/test_dp_overlap.py tests/gpu/test_native_runtime.py tests/gpu/test_launch_list.py \
  tests/gpu/test_p2p.py tests/kernels/test_amp.py tests/kernels/test_iconv.py tests/kernels/test_norm.py tests/gpu/test_model_parity.py \
  > gpurun_out/r3_dp_tests.log 2>&1 || { tail -40 gpurun_out/r3_dp_tests.log; exit 1; }
tail -3 gpurun_out/r3_dp_tests.log
timeout -k 10 120 python bench/graph_branch_probe.py > gpurun_out/r3_branch_probe.json 2>gpurun_out/r3_branch_probe.err || exit 1
cat gpurun_out/r3_branch_probe.json
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_lenet.json 2>gpurun_out/r3_lenet.err || exit 1
cat gpurun_out/r3_lenet.json
timeout -k 10 300 python bench.py --model vit_b16 --steps 10 --warmup 3 > gpurun_out/r3_vit.json 2>gpurun_out/r3_vit.err || exit 1
cat gpurun_out/r3_vit.json
