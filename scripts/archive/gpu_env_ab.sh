#!/bin/bash
# A/B of one environment switch on the model benches: VAR=<name> VALS="a b" MODELS="resnet50 resnet18"
# [TESTS="tests/kernels/test_iconv.py"] -> gpurun_out/env_ab.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; : > gpurun_out/env_ab.jsonl
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test_ab.log 2>&1 || { tail -30 gpurun_out/test_ab.log; exit 1; }
  tail -1 gpurun_out/test_ab.log
fi
for m in ${MODELS:-resnet50 resnet18}; do
for v in $VALS $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --model $m --steps ${STEPS:-20} --warmup 3 2> gpurun_out/ab_$m.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model':'$m','$VAR':'$v','value':d['value'],'ms':d['ms_per_step'],'p50':d['step_ms_p50'],'host':d['host_ms_p50']}))" >> gpurun_out/env_ab.jsonl || exit 1
done
done
cat gpurun_out/env_ab.jsonl
