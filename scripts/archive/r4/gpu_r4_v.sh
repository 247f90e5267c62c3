#!/bin/bash
# LibLinear for heads with out_features % 8 != 0 (ResNet-18 CIFAR fc): numerics + benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/kernels/test_linear_conv.py::test_lib_linear_bias_grad" \
  tests/kernels/test_ce_optim.py tests/kernels/test_fp16.py tests/gpu/test_model_parity.py tests/gpu/test_launcher_gpu.py > gpurun_out/r4v_tests.log 2>&1 || { tail -30 gpurun_out/r4v_tests.log; exit 1; }
tail -2 gpurun_out/r4v_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r4v_rn18.json 2>/dev/null || exit 1
  echo "rn18 $(python3 -c "import json;r=json.loads(open('gpurun_out/r4v_rn18.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
  timeout -k 10 300 python bench.py --model resnet18 --mp fp16 --steps 20 --warmup 5 > gpurun_out/r4v_rn18h.json 2>/dev/null || exit 1
  echo "rn18 fp16 $(python3 -c "import json;r=json.loads(open('gpurun_out/r4v_rn18h.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
done
