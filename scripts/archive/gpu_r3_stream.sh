#!/bin/bash
# streamed-query fused attention backward: numerics (all three backward kernels) + probe + ViT A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -x -q -k attention --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/stream_tests.log 2>&1 || { tail -30 gpurun_out/stream_tests.log; exit 1; }
tail -1 gpurun_out/stream_tests.log
timeout -k 10 120 python -u bench/attn_probe.py > gpurun_out/stream_probe.json 2> gpurun_out/stream_probe.err || exit 1
cat gpurun_out/stream_probe.json
for mode in fused stream; do
  ROCKET_ATTN_BWD=$mode timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/stream_vit_$mode.json 2> gpurun_out/stream_vit.err || exit 1
  python -c "import json;r=json.load(open('gpurun_out/stream_vit_$mode.json'));print('$mode',r['value'],r['ms_per_step'])"
done
