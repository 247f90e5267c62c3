#!/bin/bash
# round 5: conv tile stores nontemporal (ROCKET_CONV_NT) A/B on ResNet-50 / ResNet-18, conv tests first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5cnt; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_iconv.py tests/kernels/test_fp16.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for pass in 1 2; do
  for nt in 0 1; do
    for m in resnet50 resnet18; do
      ROCKET_CONV_NT=$nt timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/${m}_${nt}_$pass.json 2>> $O/err.log || exit 1
      python3 -c "import json;r=json.loads(open('$O/${m}_${nt}_$pass.json').read().strip().splitlines()[-1]);print('$m nt=$nt pass=$pass', r['value'], r['ms_per_step'])"
    done
  done
done
