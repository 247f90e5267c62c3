#!/bin/bash
# round 5: fp16 LeNet, scheduler light snapshot on / off, alternating, 3 passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5fp; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for pass in 1 2 3; do
  for l in 1 0; do
    ROCKET_SCHED_LIGHT=$l timeout -k 10 120 python bench.py --mp fp16 > $O/fp_${l}_$pass.json 2>> $O/err.log || exit 1
    python3 -c "import json;r=json.loads(open('$O/fp_${l}_$pass.json').read().strip().splitlines()[-1]);print('light=$l pass=$pass', r['value'], r['ms_per_step'], r['step_ms_p50'], r['host_issue_ms'])"
  done
done
