#!/bin/bash
# ViT-B/16 steady-state kernel traces under two GEMM routings -> gpurun_out/vit_kernels_{lib,native}.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for mode in lib native; do
  cd /tmp && ROCKET_VIT_GEMM=$mode timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_vit_$mode -o run -- python3 $R/bench.py --model vit_b16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vit_$mode.log 2>&1 || exit 1
  cd $R && f=$(find gpurun_out/prof_vit_$mode -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "ViT-B/16 bf16 bs128, ROCKET_VIT_GEMM=$mode - rocprofv3 --kernel-trace" > gpurun_out/vit_kernels_$mode.md || exit 1
  rm -rf gpurun_out/prof_vit_$mode
done
