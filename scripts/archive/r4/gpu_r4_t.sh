#!/bin/bash
# native patchify: numerics + ViT benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/kernels/test_mgemm.py::test_patchify_kernel_is_the_im2col_permutation" \
  "tests/kernels/test_mgemm.py::test_patch_embed_matches_conv" tests/kernels/test_fp16_vit.py > gpurun_out/r4t_tests.log 2>&1 || { tail -30 gpurun_out/r4t_tests.log; exit 1; }
tail -2 gpurun_out/r4t_tests.log
for i in 1 2; do
for mp in bf16 fp16; do
  timeout -k 10 300 python bench.py --model vit_b16 --mp $mp --steps 20 --warmup 5 > gpurun_out/r4t_vit_$mp.json 2>/dev/null || exit 1
  echo "vit $mp $(python3 -c "import json;r=json.loads(open('gpurun_out/r4t_vit_$mp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
done
done
