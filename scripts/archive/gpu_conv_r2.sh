#!/bin/bash
# ResNet conv path: conv tests, then ResNet-18/50 benches (one JSON line each) -> gpurun_out/resnet_r2.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; : > gpurun_out/resnet_r2.jsonl
timeout -k 10 400 python -u -m pytest tests/kernels/test_iconv.py tests/kernels/test_norm.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test_conv.log 2>&1
rc=$?; tail -3 gpurun_out/test_conv.log; [ $rc -eq 0 ] || exit $rc
for m in ${MODELS:-resnet18 resnet50}; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 2> gpurun_out/bench_$m.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model':'$m','value':d['value'],'ms':d['ms_per_step'],'p50':d['step_ms_p50'],'host':d['host_ms_p50']}))" >> gpurun_out/resnet_r2.jsonl || exit 1
done
cat gpurun_out/resnet_r2.jsonl
