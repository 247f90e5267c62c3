#!/bin/bash
# round 5: LeNet staging phase with the step's own row gather (default) vs a pre-gathered batch
# (ROCKET_DEFER_GATHER=0: a gather launch per step, the train kernel reads the batch directly)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5dg; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for d in 1 0; do
  ROCKET_DEFER_GATHER=$d ROCKET_LENET_TRACE=$O/tl_$d.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/b_$d.json 2>>$O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/tl_$d.json')); s=d['spans']
print('defer=$d', json.dumps(s)[:600])
for p in d['fwd_phases'][:3]: print(p['phase'], p['median_us_since_prev'])"
done
