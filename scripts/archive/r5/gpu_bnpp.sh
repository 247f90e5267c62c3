#!/bin/bash
# round 5: software-pipelined BatchNorm elementwise passes (ROCKET_BN_EW bit 2: 5 = pipelined +
# nontemporal on >= 64 MB tensors) vs the default (1): BN tests, fused-BN probe, ResNet-50 / -18
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5bnpp; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
ROCKET_BN_EW=5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py tests/kernels/test_iconv.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for ev in 1 5; do
  ROCKET_BN_EW=$ev timeout -k 10 200 python bench/bn_probe.py > $O/probe_$ev.jsonl 2>> $O/err.log || exit 1
  echo "probe ev=$ev"; cut -c1-120 $O/probe_$ev.jsonl
done
for pass in 1 2; do
  for ev in 1 5; do
    ROCKET_BN_EW=$ev timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${ev}_$pass.json 2>> $O/err.log || exit 1
    ROCKET_BN_EW=$ev timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/r18_${ev}_$pass.json 2>> $O/err.log || exit 1
    for f in r50_${ev}_$pass r18_${ev}_$pass; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'])"; done
  done
done
