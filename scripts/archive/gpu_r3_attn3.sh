#!/bin/bash
# fused attention backward (unrolled dQ chain, branch-free softmax gradient) + conv wgrad PMC
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_norm.py -x -q -k attention --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn3_tests.log 2>&1 || { tail -30 gpurun_out/attn3_tests.log; exit 1; }
tail -1 gpurun_out/attn3_tests.log
timeout -k 10 120 python -u bench/attn_probe.py > gpurun_out/attn3_probe.json 2> gpurun_out/attn3_probe.err || exit 1
cat gpurun_out/attn3_probe.json
timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/attn3_vit.json 2> gpurun_out/attn3_vit.err || exit 1
python -c "import json;r=json.load(open('gpurun_out/attn3_vit.json'));print('vit',r['value'],r['ms_per_step'])"
bash scripts/gpu_r3_wgpmc.sh
