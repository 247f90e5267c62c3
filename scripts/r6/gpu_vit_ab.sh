#!/bin/bash
# ViT-B/16 in-model A/B over env settings: VARIANTS="name:ENV=V,ENV2=V2 ..." -> one line each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6ab; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for v in $VARIANTS; do
  n=${v%%:*}; e=${v#*:}; e=${e//,/ }
  env $e timeout -k 10 300 python bench.py --model vit_b16 --steps ${STEPS:-20} --warmup 5 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;r=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print('vit $n', r['value'], r['ms_per_step'])"
done
