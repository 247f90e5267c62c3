#!/bin/bash
# round 5: ResNet-18 (CIFAR shape) with the BN elementwise / conv-store nontemporal knobs on and off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5r18; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for pass in 1 2; do
  for cfg in "1 1" "0 1" "1 0" "0 0"; do
    set -- $cfg
    ROCKET_BN_EW=$1 ROCKET_CONV_NT=$2 timeout -k 10 300 python bench.py --model resnet18 --steps 30 --warmup 5 > $O/r18_$1$2_$pass.json 2>> $O/err.log || exit 1
    python3 -c "import json;r=json.loads(open('$O/r18_$1$2_$pass.json').read().strip().splitlines()[-1]);print('r18 bn_ew=$1 conv_nt=$2 pass=$pass', r['value'], r['ms_per_step'])"
  done
done
