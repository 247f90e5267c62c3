#!/bin/bash
# native global-average-pool head + LibLinear fc for ResNet; fp16 PatchEmbed: numerics + benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_pool.py \
  "tests/kernels/test_mgemm.py::test_patch_embed_matches_conv" tests/kernels/test_fp16_vit.py tests/kernels/test_fp16.py \
  tests/gpu/test_model_parity.py tests/gpu/test_launcher_gpu.py > gpurun_out/r4r_tests.log 2>&1 || { tail -30 gpurun_out/r4r_tests.log; exit 1; }
tail -2 gpurun_out/r4r_tests.log
for m in resnet50 resnet18 vit_b16; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r4r_$m.json 2>/dev/null || exit 1
  echo "$m $(python3 -c "import json;r=json.loads(open('gpurun_out/r4r_$m.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --model vit_b16 --mp fp16 --steps 20 --warmup 5 > gpurun_out/r4r_vit16.json 2>/dev/null || exit 1
echo "vit16 $(python3 -c "import json;r=json.loads(open('gpurun_out/r4r_vit16.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r4r_resnet18b.json 2>/dev/null || exit 1
echo "resnet18 $(python3 -c "import json;r=json.loads(open('gpurun_out/r4r_resnet18b.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
