#!/bin/bash
# Ping-pong GEMM (tile 10): numerics tests, then the per-shape probe against tile 0 and hipBLASLt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_mgemm.py -k pingpong -x -q --timeout 120 --timeout-method thread > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -2 gpurun_out/pp_tests.log
timeout -k 10 300 python -u bench/mgemm_pp_probe.py --tiles ${TILES:-0,10} > gpurun_out/pp_probe.log 2>&1; rc=$?
cat gpurun_out/pp_probe.log
exit $rc
