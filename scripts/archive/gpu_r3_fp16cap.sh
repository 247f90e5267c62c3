#!/bin/bash
# fp16 steps captured as graphs: launcher/amp GPU tests, then fp16 benches (lenet, resnet18, resnet50, vit)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_launcher_gpu.py tests/kernels/test_amp.py -m gpu > gpurun_out/fp16cap_tests.log 2>&1 || { tail -40 gpurun_out/fp16cap_tests.log; exit 1; }
tail -2 gpurun_out/fp16cap_tests.log
for m in lenet resnet18 resnet50 vit_b16; do
  timeout -k 10 300 python bench.py --model $m --mp fp16 --steps 20 --warmup 5 > gpurun_out/fp16cap_$m.json 2> gpurun_out/fp16cap_$m.err || { tail -20 gpurun_out/fp16cap_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fp16cap_$m.json'));print('$m',d['value'],d['ms_per_step'],d['host_issue_ms'])"
done
