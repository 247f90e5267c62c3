#!/bin/bash
# round 5 box o: same-box A/B of the attention dQ pipelining (ab_old = HEAD library): probe + ViT bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5o; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for v in new old new old; do
  if [ $v = old ]; then export ROCKET_LIBDIR=$R/ab_old; else unset ROCKET_LIBDIR; fi
  timeout -k 10 120 python bench/attn_probe.py > $O/probe_$v.json 2>> $O/err.log || exit 1
  echo "$v $(cat $O/probe_$v.json)"
  timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_$v.json 2>> $O/err.log || exit 1
  python3 -c "import json;r=json.loads(open('$O/vit_$v.json').read().strip().splitlines()[-1]);print('vit $v', r['value'], r['ms_per_step'])"
done
