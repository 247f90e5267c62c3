#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py tests/gpu/test_model_parity.py > gpurun_out/r3_vit_tests.log 2>&1 || { tail -30 gpurun_out/r3_vit_tests.log; exit 1; }
tail -2 gpurun_out/r3_vit_tests.log
for m in lib libw native; do
  ROCKET_VIT_GEMM=$m timeout -k 10 300 python bench.py --model vit_b16 --steps 10 --warmup 3 > gpurun_out/r3_vit_$m.json 2>gpurun_out/r3_vit_$m.err || exit 1
  echo "$m: $(python -c "import json;d=json.load(open('gpurun_out/r3_vit_$m.json'));print(d['value'], d['ms_per_step'])")"
done
