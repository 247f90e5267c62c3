#!/bin/bash
# ViT-B/16 steady-state kernel trace summary -> gpurun_out/vit_kernels.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_vit -o run -- python3 $R/bench.py --model vit_b16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vit.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/prof_vit -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "ViT-B/16 224^2 bf16 bs128, 1x MI355X - rocprofv3 --kernel-trace" > gpurun_out/vit_kernels.md; rc=$?
rm -rf gpurun_out/prof_vit
exit $rc
