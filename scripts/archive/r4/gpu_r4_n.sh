#!/bin/bash
# engine-level fp16 fused LeNet test
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_launcher_gpu.py > gpurun_out/r4n_tests.log 2>&1 || { tail -40 gpurun_out/r4n_tests.log; exit 1; }
tail -12 gpurun_out/r4n_tests.log
bash scripts/archive/r4/gpu_r4_o.sh
