#!/bin/bash
# round 5: ROCKET_SCHED_LIGHT 0 vs 1 with the queued provisional steps (fp16 LeNet)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5sl; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_fp16.py tests/unit/test_sched_speculation.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for pass in 1 2; do
  for q in 0 1; do
    ROCKET_SCHED_LIGHT=$q timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --mp fp16 > $O/drv_${q}_$pass.json 2>> $O/err.log || exit 1
    ROCKET_SCHED_LIGHT=$q timeout -k 10 120 python bench.py --steps 1000 --warmup 50 --mp fp16 > $O/long_${q}_$pass.json 2>> $O/err.log || exit 1
    for f in drv_${q}_$pass long_${q}_$pass; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'], r.get('host_issue_ms'))"; done
  done
done
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bf16.json 2>> $O/err.log || exit 1
python3 -c "import json;r=json.loads(open('$O/bf16.json').read().strip().splitlines()[-1]);print('bf16', r['value'], r['ms_per_step'], r['step_ms_p50'])"
