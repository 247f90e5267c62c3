#!/bin/bash
# current LeNet captured-step phase timeline (fused train kernel + wgrad kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3t; export TMPDIR=/tmp
O=$R/gpurun_out/r3t
ROCKET_LENET_TRACE=$O/trace_now.json timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/traced.json 2>$O/traced.err || { tail -20 $O/traced.err; exit 1; }
python - <<PY
import json
d=json.load(open('$O/trace_now.json'))
print(json.dumps(d['spans']))
for k in d:
    if k.endswith('phases'):
        print(k)
        for p in d[k]: print('   %-40s %6.2f %6.2f'%(p['phase'],p['median_us_since_prev'],p['median_us_since_launch']))
PY
