#!/bin/bash
# Selected GPU tests: ${TESTS} (default: kernel + graph-capture tests)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/kernels tests/gpu/test_graph_capture.py} -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1; rc=$?
echo "pytest rc=$rc" > gpurun_out/summary_quick.txt
exit $rc
