#!/bin/bash
# round 6 box b: persistent GEMM (xgemm5) numerics + probe vs hipBLASLt / xgemm4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6b; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/kernels/test_xgemm5.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python bench/gemm_r6_probe.py --out $O/probe.jsonl > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.jsonl
