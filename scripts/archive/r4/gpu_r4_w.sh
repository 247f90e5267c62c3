#!/bin/bash
# LibLinear wgrad fallback for unaligned flat-bucket grads: DDP rehearsals + LibLinear numerics
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/gpu/test_ddp_graph.py \
  "tests/kernels/test_linear_conv.py::test_lib_linear_bias_grad" tests/gpu/test_multigpu.py tests/gpu/test_model_parity.py > gpurun_out/r4w_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r4w_tests.log
exit $rc
