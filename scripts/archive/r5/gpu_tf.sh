#!/bin/bash
# round 5: fp16 LeNet step timeline + kernel trace (what the extra fp16 GPU time is)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5tf; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
ROCKET_LENET_TRACE=$O/tl.json timeout -k 10 120 python bench.py --mp fp16 --steps 200 --warmup 20 > $O/tl_b.json 2>>$O/err.log || exit 1
python3 -c "
import json; d=json.load(open('$O/tl.json')); s=d['spans']
print(json.dumps(s)[:900])
for p in d['fwd_phases']+d['bwd_phases']: print(p['phase'], p['median_us_since_prev'])"
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/bench.py --mp fp16 --steps 200 --warmup 20 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
cd $R && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cat {} | head -20
