#!/bin/bash
# fp16 ViT-B/16 kernel trace (after the fp16 GEMM table)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4q_vit16 -o run -- python3 $R/bench.py --model vit_b16 --mp fp16 --steps 8 --warmup 3 > $R/gpurun_out/r4q_trace.log 2>&1 || { tail -20 $R/gpurun_out/r4q_trace.log; exit 1; }
cd $R
f=$(find gpurun_out/r4q_vit16 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ViT-B/16 bs128 fp16 step (round 4), rocprofv3 kernel trace" > gpurun_out/r4_vit_b16_fp16_kernels.md
rm -rf gpurun_out/r4q_vit16
head -40 gpurun_out/r4_vit_b16_fp16_kernels.md
bash scripts/archive/r4/gpu_r4_pmc.sh
