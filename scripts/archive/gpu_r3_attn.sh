#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/kernels/test_norm.py -k attention > gpurun_out/r3_attn_test.log 2>&1 || { tail -30 gpurun_out/r3_attn_test.log; exit 1; }
tail -2 gpurun_out/r3_attn_test.log
timeout -k 10 120 python bench/attn_probe.py > gpurun_out/r3_attn_probe.json 2>&1 || exit 1
cat gpurun_out/r3_attn_probe.json
