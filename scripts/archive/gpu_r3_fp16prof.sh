#!/bin/bash
# kernel traces of the captured fp16 steps (ResNet-18, ViT-B/16)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${PROF_MODELS:-resnet18 vit_b16}; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof16_$m -o run -- python3 $R/bench.py --model $m --mp fp16 --steps 6 --warmup 3 > $R/gpurun_out/prof16_$m.log 2>&1 || exit 1
  cd $R && f=$(find gpurun_out/prof16_$m -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "$m fp16 (captured step, device GradScaler) - rocprofv3 --kernel-trace (round 3)" > gpurun_out/kernels16_$m.md || exit 1
  head -5 gpurun_out/kernels16_$m.md
done
