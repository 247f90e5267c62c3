#!/bin/bash
# round 6 final confirmation on a rebuilt tree: GPU suite, smoke(), then the bench set (gpu_benches.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6final; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1 \
  || { tail -60 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
bash scripts/r6/gpu_benches.sh
