#!/bin/bash
# end-of-round kernel traces: ViT-B/16 bf16, ResNet-18 bf16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4u_vit -o run -- python3 $R/bench.py --model vit_b16 --steps 8 --warmup 3 > $R/gpurun_out/r4u_vit.log 2>&1 || { tail -20 $R/gpurun_out/r4u_vit.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4u_rn18 -o run -- python3 $R/bench.py --model resnet18 --steps 8 --warmup 3 > $R/gpurun_out/r4u_rn18.log 2>&1 || { tail -20 $R/gpurun_out/r4u_rn18.log; exit 1; }
cd $R
f=$(find gpurun_out/r4u_vit -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ViT-B/16 bs128 bf16 step (round 4, end of round), rocprofv3 kernel trace" > gpurun_out/r4_vit_b16_kernels_end.md
f=$(find gpurun_out/r4u_rn18 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ResNet-18 bs256 bf16 step (round 4, end of round), rocprofv3 kernel trace" > gpurun_out/r4_resnet18_kernels.md
rm -rf gpurun_out/r4u_vit gpurun_out/r4u_rn18
head -5 gpurun_out/r4_vit_b16_kernels_end.md; tail -16 gpurun_out/r4_vit_b16_kernels_end.md; head -5 gpurun_out/r4_resnet18_kernels.md; tail -14 gpurun_out/r4_resnet18_kernels.md
