#!/bin/bash
# Round 3 batch: LN/bias-link + parity tests, ViT GEMM routings, ResNet-50 launch-list vs graph
# replay (host time), LeNet phase timeline + kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py tests/gpu/test_model_parity.py > gpurun_out/r3_d_tests.log 2>&1 || { tail -30 gpurun_out/r3_d_tests.log; exit 1; }
tail -2 gpurun_out/r3_d_tests.log
for m in lib libw native; do
  ROCKET_VIT_GEMM=$m timeout -k 10 300 python bench.py --model vit_b16 --steps 10 --warmup 3 > gpurun_out/r3_vit_$m.json 2>gpurun_out/r3_vit_$m.err || exit 1
  echo "vit $m: $(python -c "import json;d=json.load(open('gpurun_out/r3_vit_$m.json'));print(d['value'], d['ms_per_step'], d['host_ms_p50'])")"
done
for ll in 1 0; do
  ROCKET_LAUNCH_LIST=$ll timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3_rn50_ll$ll.json 2>gpurun_out/r3_rn50_ll$ll.err || exit 1
  echo "rn50 launchlist=$ll: $(python -c "import json;d=json.load(open('gpurun_out/r3_rn50_ll$ll.json'));print(d['value'], d['ms_per_step'], d['host_ms_p50'])")"
done
timeout -k 10 120 python bench/lenet_timeline.py > gpurun_out/r3_lenet_timeline.jsonl 2> gpurun_out/r3_lenet_timeline.err || exit 1
head -c 2500 gpurun_out/r3_lenet_timeline.jsonl
