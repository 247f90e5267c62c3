#!/bin/bash
# LeNet driver-shape A/B over env settings, interleaved: VARIANTS="name:ENV=V ..." ROUNDS=n
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6lab; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for k in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    n=${v%%:*}; e=${v#*:}; e=${e//,/ }
    env $e timeout -k 10 120 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} > $O/$n.$k.json 2> $O/$n.$k.err || { tail -20 $O/$n.$k.err; exit 1; }
    python3 -c "import json;r=json.loads(open('$O/$n.$k.json').read().strip().splitlines()[-1]);print('$n', r['value'], r['ms_per_step'], r.get('step_ms_p50'))"
  done
done
