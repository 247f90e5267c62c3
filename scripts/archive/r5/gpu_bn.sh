#!/bin/bash
# round 5: BatchNorm elementwise-pass variants (ROCKET_BN_EW: bit 0 nontemporal, bit 1 8 rows in flight):
# kernel probe (fused BN fwd+bwd, ResNet-50 shapes) and ResNet-50 / ResNet-18 step, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5bn; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for ev in 0 1 2 3; do
  ROCKET_BN_EW=$ev timeout -k 10 200 python bench/bn_probe.py > $O/probe_$ev.jsonl 2>> $O/err.log || exit 1
done
for pass in 1 2; do
  for ev in 0 1 3; do
    ROCKET_BN_EW=$ev timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${ev}_$pass.json 2>> $O/err.log || exit 1
    python3 -c "import json;r=json.loads(open('$O/r50_${ev}_$pass.json').read().strip().splitlines()[-1]);print('r50 ev=$ev pass=$pass', r['value'], r['ms_per_step'])"
  done
done
for ev in 0 1 2 3; do echo "probe ev=$ev"; cat $O/probe_$ev.jsonl; done
