#!/bin/bash
# strided conv input gradient: native parity-class launch vs library, ResNet-50 / ResNet-18
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; : > gpurun_out/sdgrad_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/kernels/test_iconv.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test_conv.log 2>&1 || { tail -20 gpurun_out/test_conv.log; exit 1; }
tail -1 gpurun_out/test_conv.log
for m in resnet50 resnet18; do
for mode in native lib native lib; do
  ROCKET_CONV_SDGRAD=$mode timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 3 2> gpurun_out/sd_$m.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model':'$m','sdgrad':'$mode','value':d['value'],'ms':d['ms_per_step'],'p50':d['step_ms_p50'],'host':d['host_ms_p50']}))" >> gpurun_out/sdgrad_ab.jsonl || exit 1
done
done
cat gpurun_out/sdgrad_ab.jsonl
