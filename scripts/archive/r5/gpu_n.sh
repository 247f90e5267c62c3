#!/bin/bash
# round 5 box n: attention backward with a software-pipelined dQ phase: tests, probe, ViT bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5n; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_fp16_vit.py tests/gpu/test_model_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python bench/attn_probe.py > $O/probe.json 2>> $O/err.log || exit 1
cat $O/probe.json
for i in 1 2; do
  timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_$i.json 2>> $O/err.log || exit 1
  python3 -c "import json;r=json.loads(open('$O/vit_$i.json').read().strip().splitlines()[-1]);print('vit', r['value'], r['ms_per_step'])"
done
