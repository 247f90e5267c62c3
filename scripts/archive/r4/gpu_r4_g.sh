#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp

timeout -k 10 300 python -u bench/xgemm4_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/xgemm4_probe.log
