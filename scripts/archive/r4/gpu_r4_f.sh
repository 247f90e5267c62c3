#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u bench/ln_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ln_probe.log
