#!/bin/bash
# BN probe, fused-vs-torch A/B for the big models, ViT kernel profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/summary_ab.txt
timeout -k 10 300 python bench/bn_probe.py > gpurun_out/bn_probe.jsonl 2> gpurun_out/bn_probe.err; echo "probe rc=$?" >> gpurun_out/summary_ab.txt
for m in resnet18 resnet50 vit_b16; do
  for impl in fused torch; do
    timeout -k 10 400 python bench.py --model $m --impl $impl --steps 20 --warmup 5 > gpurun_out/ab_${m}_${impl}.json 2> gpurun_out/ab_${m}_${impl}.err; rc=$?; echo "$m $impl rc=$rc" >> gpurun_out/summary_ab.txt
    [ $rc -ne 0 ] && exit 1
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_vit -o run -- python3 bench.py --model vit_b16 --steps 10 --warmup 3 > gpurun_out/prof_vit.log 2>&1; echo "prof rc=$?" >> gpurun_out/summary_ab.txt
