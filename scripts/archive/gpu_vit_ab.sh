#!/bin/bash
# ViT-B/16: mlinear tests, then the bench under each GEMM routing (hybrid / native / lib)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out; : > gpurun_out/vit_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/kernels/test_mgemm.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test_mgemm.log 2>&1
rc=$?; tail -2 gpurun_out/test_mgemm.log; [ $rc -eq 0 ] || exit $rc
for mode in hybrid lib native hybrid; do
  ROCKET_VIT_GEMM=$mode timeout -k 10 300 python bench.py --model vit_b16 --steps 10 --warmup 3 2> gpurun_out/vit_$mode.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'mode':'$mode','value':d['value'],'ms':d['ms_per_step'],'host':d['host_ms_p50']}))" >> gpurun_out/vit_ab.jsonl || exit 1
done
cat gpurun_out/vit_ab.jsonl
