#!/bin/bash
# conv gather address changes: conv numerics tests, per-shape probe, ResNet benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_iconv.py tests/kernels/test_fp16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gat_tests.log 2>&1 || { tail -30 gpurun_out/gat_tests.log; exit 1; }
tail -2 gpurun_out/gat_tests.log
timeout -k 10 300 python -u bench/iconv_probe.py --model resnet50 --cfgs 0 > gpurun_out/gat2_rn50.jsonl 2> gpurun_out/gat2_rn50.err || exit 1
timeout -k 10 200 python -u bench/iconv_probe.py --model resnet18 --cfgs 0 > gpurun_out/gat2_rn18.jsonl 2> gpurun_out/gat2_rn18.err || exit 1
grep cfg gpurun_out/gat2_rn50.jsonl gpurun_out/gat2_rn18.jsonl
for m in resnet18 resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/gat2_$m.json 2> gpurun_out/gat2_$m.err || exit 1
  python -c "import json;r=json.load(open('gpurun_out/gat2_$m.json'));print('$m',r['value'],r['ms_per_step'])"
done
