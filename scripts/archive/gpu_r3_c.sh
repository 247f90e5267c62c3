#!/bin/bash
# Round 3: attention probe, graph-branch concurrency (both packet-capture modes), ResNet-50 conv
# per-shape probe, ViT A/B (fused vs split attention backward) + kernel trace, LeNet variance
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python bench/attn_probe.py > gpurun_out/r3_attn_probe.json 2>&1 || exit 1
cat gpurun_out/r3_attn_probe.json
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python bench/graph_branch_probe.py > gpurun_out/r3_branch_pc0.json 2>&1 || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 python bench/graph_branch_probe.py > gpurun_out/r3_branch_pc1.json 2>&1 || exit 1
cat gpurun_out/r3_branch_pc0.json gpurun_out/r3_branch_pc1.json
for a in fused split; do
  ROCKET_ATTN_BWD=$a timeout -k 10 300 python bench.py --model vit_b16 --steps 10 --warmup 3 > gpurun_out/r3_vit_$a.json 2>gpurun_out/r3_vit_$a.err || exit 1
  cat gpurun_out/r3_vit_$a.json
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_lenet_$i.json 2>&1 || exit 1
  cat gpurun_out/r3_lenet_$i.json
done
timeout -k 10 300 python bench/iconv_probe.py --model resnet50 > gpurun_out/r3_iconv_rn50.jsonl 2>&1 || exit 1
tail -3 gpurun_out/r3_iconv_rn50.jsonl
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_vit -o run -- python3 $R/bench.py --model vit_b16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vit.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/prof_vit -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "ViT-B/16 224^2 bf16 bs128, 1x MI355X - rocprofv3 --kernel-trace" > gpurun_out/r3_vit_kernels.md; rc=$?
rm -rf gpurun_out/prof_vit
head -30 gpurun_out/r3_vit_kernels.md
exit $rc
