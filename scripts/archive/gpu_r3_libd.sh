#!/bin/bash
# ViT GEMM routing A/B: lib vs libd (native input gradients, gelu' in fc2's dgrad epilogue) vs native
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_mgemm.py -x -q -k "mlinear or mmlp or direct" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/libd_tests.log 2>&1 || { tail -30 gpurun_out/libd_tests.log; exit 1; }
tail -1 gpurun_out/libd_tests.log
for rep in 1 2; do
for mode in lib libd native; do
  ROCKET_VIT_GEMM=$mode timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/libd_$mode.json 2> gpurun_out/libd_$mode.err || exit 1
  python -c "import json;r=json.load(open('gpurun_out/libd_$mode.json'));print('$mode',r['value'],r['ms_per_step'])"
done
done
