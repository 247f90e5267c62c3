#!/bin/bash
# big models with and without HIP-graph capture of the step
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out; : > gpurun_out/graph_models.jsonl
for model in resnet18 resnet50 vit_b16; do
  for g in "" "--graph"; do
    timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 3 $g 2> gpurun_out/gm_${model}$g.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model':'$model','graph':'$g','value':d['value'],'ms':d['ms_per_step'],'p50':d['step_ms_p50'],'host':d['host_ms_p50']}))" >> gpurun_out/graph_models.jsonl || { echo "$model $g failed" >> gpurun_out/graph_models.jsonl; tail -3 gpurun_out/gm_${model}$g.err >> gpurun_out/graph_models.jsonl; }
  done
done
cat gpurun_out/graph_models.jsonl
