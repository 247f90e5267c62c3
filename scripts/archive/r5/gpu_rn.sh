#!/bin/bash
# round 5: ResNet-18 / ResNet-50 at HEAD defaults, twice each, plus the BN numerics tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5rn; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py tests/kernels/test_iconv.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for pass in 1 2; do
  for m in resnet18 resnet50; do
    timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/${m}_$pass.json 2>> $O/err.log || exit 1
    python3 -c "import json;r=json.loads(open('$O/${m}_$pass.json').read().strip().splitlines()[-1]);print('$m pass=$pass', r['value'], r['ms_per_step'])"
  done
done
