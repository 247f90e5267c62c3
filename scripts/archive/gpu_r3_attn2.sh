#!/bin/bash
# attention staging + conv gather address changes: numerics tests, probes, model benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_norm.py tests/kernels/test_iconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn2_tests.log 2>&1 || { tail -30 gpurun_out/attn2_tests.log; exit 1; }
tail -2 gpurun_out/attn2_tests.log
timeout -k 10 120 python -u bench/attn_probe.py > gpurun_out/attn2_probe.json 2> gpurun_out/attn2_probe.err || exit 1
cat gpurun_out/attn2_probe.json
timeout -k 10 300 python -u bench/iconv_probe.py --model resnet50 --cfgs 0 > gpurun_out/gat_rn50.jsonl 2> gpurun_out/gat_rn50.err || exit 1
timeout -k 10 200 python -u bench/iconv_probe.py --model resnet18 --cfgs 0 > gpurun_out/gat_rn18.jsonl 2> gpurun_out/gat_rn18.err || exit 1
grep cfg gpurun_out/gat_rn50.jsonl gpurun_out/gat_rn18.jsonl
for m in resnet18 resnet50 vit_b16; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/attn2_$m.json 2> gpurun_out/attn2_$m.err || exit 1
  cat gpurun_out/attn2_$m.json
done
ROCKET_VIT_GEMM=libw timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/attn2_vit_libw.json 2> gpurun_out/attn2_vit_libw.err || exit 1
cat gpurun_out/attn2_vit_libw.json
