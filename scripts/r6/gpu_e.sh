#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6e; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 200 python bench/x5_diag.py > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
grep -v amdgpu.ids $O/diag.log | cut -c1-330
