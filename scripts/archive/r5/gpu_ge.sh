#!/bin/bash
# round 5: GELU passes (ROCKET_GELU_EW: 0 = 4-element kernels, 2 = 16-byte nontemporal forward and
# nontemporal GELU-backward+colsum): tests, then ViT-B/16 bf16 alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ge; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_fp16_vit.py tests/kernels/test_mgemm.py tests/kernels/test_norm.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for pass in 1 2; do
  for ev in 0 2; do
    ROCKET_GELU_EW=$ev timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_${ev}_$pass.json 2>> $O/err.log || exit 1
    python3 -c "import json;r=json.loads(open('$O/vit_${ev}_$pass.json').read().strip().splitlines()[-1]);print('vit ev=$ev pass=$pass', r['value'], r['ms_per_step'])"
  done
done
