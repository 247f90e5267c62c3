#!/bin/bash
# ResNet-18 / ResNet-50 bench under ROCKET_CONV=native vs lib (MIOpen)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out; : > gpurun_out/resnet_ab.jsonl
for model in resnet50 resnet18; do
  for mode in native lib; do
    ROCKET_CONV=$mode timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 3 2> gpurun_out/rn_${model}_$mode.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model':'$model','mode':'$mode','value':d['value'],'ms':d['ms_per_step'],'host':d['host_ms_p50']}))" >> gpurun_out/resnet_ab.jsonl || { tail -5 gpurun_out/rn_${model}_$mode.err; exit 1; }
  done
done
cat gpurun_out/resnet_ab.jsonl
