#!/bin/bash
# round 5 (end): full GPU test suite + smoke at HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/suite_pytest.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/suite_pytest.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite_smoke.log 2>&1 && echo "smoke ok"
