#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_r4_c.sh && bash scripts/gpu_r4_d.sh
