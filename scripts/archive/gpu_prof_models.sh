#!/bin/bash
# Steady-state kernel traces of the bench models -> gpurun_out/kernels_<model>.md
# usage: MODELS="vit_b16 resnet18" bash scripts/gpu_prof_models.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${MODELS:-vit_b16}; do
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_$m -o run -- python3 $R/bench.py --model $m --steps 5 --warmup 2 > $R/gpurun_out/prof_$m.log 2>&1 || exit 1
  cd $R && f=$(find gpurun_out/prof_$m -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "$m bf16 - rocprofv3 --kernel-trace (HEAD $(cat .head 2>/dev/null))" > gpurun_out/kernels_$m.md || exit 1
  rm -rf gpurun_out/prof_$m
done
