#!/bin/bash
# round-6 bench set: LeNet driver shape x2, LeNet 1000 steps, fp16 LeNet, ResNet-18/50, ViT-B/16 (bf16 default
# route, fp16) -> gpurun_out/r6bench/summary.txt (one line per run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6bench; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
run() {  # tag, timeout, args...
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -20 $O/$tag.err; return 1; }
  python3 -c "import json;r=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);print('$tag', r['value'], r['unit'], r['ms_per_step'], r.get('step_ms_p50'), r.get('host_issue_ms'))" | tee -a $O/summary.txt
}
run lenet_drv1 120 --gpus 1 --steps 20 --warmup 5 &&
run lenet_drv2 120 --gpus 1 --steps 20 --warmup 5 &&
run lenet_long 180 --gpus 1 --steps 1000 --warmup 50 &&
run lenet_fp16 180 --gpus 1 --steps 1000 --warmup 50 --mp fp16 &&
run resnet18 400 --model resnet18 --steps 20 --warmup 5 &&
run resnet50 400 --model resnet50 --steps 20 --warmup 5 &&
run vit_b16 400 --model vit_b16 --steps 20 --warmup 5 &&
run vit_b16_fp16 400 --model vit_b16 --steps 20 --warmup 5 --mp fp16
