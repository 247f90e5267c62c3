#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/dbg/lenet_fp16_grads.py 2>&1 | tee gpurun_out/r4_dbg.log
