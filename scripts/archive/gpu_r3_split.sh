#!/bin/bash
# wgrad split-K model rate A/B (ROCKET_WGRAD_RATE_CU) on ResNet-18 / ResNet-50
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for rate in 3.5e12 1.2e12 1e13; do
  for m in resnet18 resnet50; do
    ROCKET_WGRAD_RATE_CU=$rate timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/split_$m.json 2> gpurun_out/split_$m.err || exit 1
    python -c "import json;r=json.load(open('gpurun_out/split_$m.json'));print('$rate $m',r['value'],r['ms_per_step'])"
  done
done
done
